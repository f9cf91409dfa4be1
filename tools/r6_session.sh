# round-6 GPU session: tests, an A/B of library variants, bench lines
#   bash tools/r6_session.sh <tag> "<test files>" "<ab variants>" "<bench configs>"
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
if [ -n "$AB" ]; then
  timeout -k 10 600 python -u tools/diag_ab.py run $AB > $OUT/ab.log 2>&1
  rc=$?; echo "ab rc=$rc"; cat $OUT/ab.log | grep variant
  [ $rc -eq 0 ] || exit $rc
fi
for C in $CONFS; do
  timeout -k 10 400 python -u bench.py --config $C --steps 20 --warmup 3 > $OUT/bench_$C.json 2> $OUT/bench_$C.err
  rc=$?; echo "bench $C rc=$rc"; cut -c1-200 $OUT/bench_$C.json
  [ $rc -eq 0 ] || exit $rc
done
