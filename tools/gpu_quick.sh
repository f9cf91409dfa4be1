# A focused GPU call: selected -m gpu test files, then bench lines of the
# given configs, then (optional) a rocprof kernel trace of one config.
#   bash tools/gpu_quick.sh <tag> "<test files>" "<configs>" [trace-config]
# Every GPU step has its own time limit; a crash / abort / timeout ends it.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=$1; TESTS=$2; CONFS=$3; TRACE=$4
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -v --tb=short --timeout 150 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest.log
  [ $rc -eq 0 ] || { echo FAILED > $OUT/FAILED; exit $rc; }
fi
for C in $CONFS; do
  NAME=${C%%:*}; EXTRA=${C#*:}; [ "$EXTRA" = "$C" ] && EXTRA=""
  TAGC=$NAME$(echo "$EXTRA" | tr -d ' -')
  timeout -k 10 400 python -u bench.py --config $NAME --steps 20 --warmup 3 $EXTRA > $OUT/bench_$TAGC.json 2> $OUT/bench_$TAGC.err
  rc=$?; echo "bench $C rc=$rc"; cut -c1-300 $OUT/bench_$TAGC.json
  [ $rc -eq 0 ] || exit $rc
done
if [ -n "$TRACE" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --config $TRACE --steps 10 --warmup 2 --no-cpu-baseline > $OUT/trace_bench.json 2> $OUT/trace_bench.err
  rc=$?; echo "trace rc=$rc"
  exit $rc
fi
