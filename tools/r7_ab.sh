# round-7-style session: GPU tests, then the same A/B over several workloads
#   bash tools/r7_ab.sh <tag> "<test files>" "<variants>" "<configs>"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=$1; TESTS=$2; AB=$3; CONFS=$4
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v --tb=short --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
for C in $CONFS; do
  CGPU_AB_CONFIG=$C timeout -k 10 600 python -u tools/diag_ab.py run $AB > $OUT/ab_$C.log 2>&1
  rc=$?; echo "ab $C rc=$rc"; grep variant $OUT/ab_$C.log
  [ $rc -eq 0 ] || exit $rc
done
