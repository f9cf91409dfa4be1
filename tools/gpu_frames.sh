# GPU session for the raw-frame row: frame parity tests,
# the whole gpu suite, smoke, and the headline + frames bench lines.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
stop() { echo "stopping: $1 rc=$2"; exit $2; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_frames.log 2>&1
rc=$?; echo "frames pytest rc=$rc"; tail -5 gpurun_out/pytest_frames.log; [ $rc = 0 ] || stop frames $rc
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "gpu pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || stop gpu $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc = 0 ] || stop smoke $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench_gpu.json 2> gpurun_out/bench_gpu.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_gpu.json; [ $rc = 0 ] || stop bench $rc
timeout -k 10 300 python -u bench.py --config frames --steps 10 --warmup 3 > gpurun_out/bench_frames.json 2> gpurun_out/bench_frames.err
rc=$?; echo "bench frames rc=$rc"; cat gpurun_out/bench_frames.json; [ $rc = 0 ] || stop bench_frames $rc
