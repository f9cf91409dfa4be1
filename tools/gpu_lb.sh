# LB row iteration: LB parity tests, then the cascade bench (config 5)
#   bash tools/gpu_lb.sh [prof]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
stop() { echo "stopping: $1 rc=$2"; exit $2; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_lb.py -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_lb.log 2>&1
rc=$?; echo "lb pytest rc=$rc"; tail -5 gpurun_out/pytest_lb.log; [ $rc = 0 ] || stop lb $rc
timeout -k 10 400 python -u bench.py --config cascade --steps 10 --warmup 3 > gpurun_out/bench_cascade.json 2> gpurun_out/bench_cascade.err
rc=$?; echo "cascade rc=$rc"; cat gpurun_out/bench_cascade.json; [ $rc = 0 ] || { tail -20 gpurun_out/bench_cascade.err; stop cascade $rc; }
if [ "${1:-}" = "prof" ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cascade -o run -- python3 bench.py --config cascade --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_cascade_bench.json 2> gpurun_out/prof_cascade_bench.err
rc=$?; echo "prof rc=$rc"; [ $rc = 0 ] || stop prof $rc
fi
