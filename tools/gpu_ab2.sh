set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
[ -n "$SKIP_TESTS" ] || timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/ab_classify.py --rounds 3 --iters 3 --configs "${AB_CONFIGS:-3:1,8:1,7:1,22:1}" > gpurun_out/ab2.json 2> gpurun_out/ab2.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab2.json
