set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log; case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 400 python -u tools/ab_classify.py --rounds 3 --iters 3 --configs "${AB_CONFIGS:-3:1,3:4,3:1:12,3:1:50,0:1,9:1}" > gpurun_out/ab.json 2> gpurun_out/ab.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab.json
