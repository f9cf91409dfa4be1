# One GPU session on the box (run from the repo root via gpurun):
#   bash tools/gpu_run.sh <tag> [pytest-args...]
# -> gpurun_out/<tag>/{pytest.log, bench.json, bench.err}
# Every GPU step has its own time limit; a crash / abort / timeout ends the
# session (no further GPU step), an ordinary test failure does not stop the
# bench that follows.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-run}
shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread "$@" > $OUT/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?
echo "smoke rc=$rc"; tail -2 $OUT/smoke.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench.json 2> $OUT/bench.err
rc=$?
echo "bench rc=$rc"; cat $OUT/bench.json
exit $rc
