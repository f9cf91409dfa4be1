# Round-5 GPU session: selected -m gpu test files, then bench lines, then
# timing-only A/Bs of diagnostic builds.
#   bash tools/r5_session.sh <tag> "<test files>" "<configs>" "<ab config>:<variants>" ...
# Every GPU step has its own time limit; a failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=$1; TESTS=$2; CONFS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v --tb=short --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
  [ $rc -eq 0 ] || { echo FAILED > $OUT/FAILED; exit $rc; }
fi
for C in $CONFS; do
  NAME=${C%%:*}; EXTRA=${C#*:}; [ "$EXTRA" = "$C" ] && EXTRA=""
  TAGC=$NAME$(echo "$EXTRA" | tr -d ' -')
  timeout -k 10 400 python -u bench.py --config $NAME --steps 20 --warmup 3 $EXTRA > $OUT/bench_$TAGC.json 2> $OUT/bench_$TAGC.err
  rc=$?; echo "bench $C rc=$rc"; cut -c1-200 $OUT/bench_$TAGC.json
  [ $rc -eq 0 ] || exit $rc
done
for AB in "$@"; do
  CONF=${AB%%:*}; VARS=${AB#*:}
  CGPU_AB_CONFIG=$CONF timeout -k 10 300 python -u tools/diag_ab.py run $VARS > $OUT/ab_$CONF.log 2>&1
  rc=$?; echo "ab $CONF rc=$rc"; tail -4 $OUT/ab_$CONF.log
  [ $rc -eq 0 ] || exit $rc
done
