# L3 MapState compilation parity on the GPU
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_l3.py tests/test_gpu_ct.py -x -v --timeout 180 --timeout-method thread > gpurun_out/pytest_l3.log 2>&1
rc=$?; echo "l3 pytest rc=$rc"; tail -16 gpurun_out/pytest_l3.log; exit $rc
