# GPU session for the conntrack row: CT parity tests,
# then the whole gpu suite.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
stop() { echo "stopping: $1 rc=$2"; exit $2; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_ct.py -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_ct.log 2>&1
rc=$?; echo "ct pytest rc=$rc"; tail -30 gpurun_out/pytest_ct.log; [ $rc = 0 ] || stop ct $rc
if [ "${1:-}" = "all" ]; then
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "gpu pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || stop gpu $rc
fi
