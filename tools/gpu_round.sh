# Round check on one GPU (run on the gpurun box from the repo root):
#   bash tools/gpu_round.sh
# the whole gpu suite, smoke(), then the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
stop() { echo "stopping: $1 rc=$2"; exit $2; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "gpu pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || stop gpu $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log; [ $rc = 0 ] || stop smoke $rc
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_default.json; [ $rc = 0 ] || { tail -20 gpurun_out/bench_default.err; stop bench $rc; }
