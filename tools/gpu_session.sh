# One GPU session: the -m gpu suite, smoke, then bench lines of the given
# configs (default: the headline config 2).  Every GPU step has its own time
# limit; a crash / abort / timeout ends the session.
#   bash tools/gpu_session.sh <tag> [config[:extra-args] ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-run}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { echo FAILED > $OUT/FAILED; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"; tail -1 $OUT/smoke.log
[ $rc -eq 0 ] || { echo FAILED > $OUT/FAILED; exit $rc; }
[ $# -gt 0 ] || set -- gpu
for C in "$@"; do
  NAME=${C%%:*}; EXTRA=${C#*:}; [ "$EXTRA" = "$C" ] && EXTRA=""
  TAGC=$NAME$(echo "$EXTRA" | tr -d ' -')
  timeout -k 10 400 python -u bench.py --config $NAME --steps 20 --warmup 3 $EXTRA > $OUT/bench_$TAGC.json 2> $OUT/bench_$TAGC.err
  rc=$?; echo "bench $C rc=$rc"; cut -c1-400 $OUT/bench_$TAGC.json
  [ $rc -eq 0 ] || exit $rc
done
