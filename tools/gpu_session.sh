# One GPU session: gpu tests, smoke, bench, interleaved A/B of classify variants.
# usage (from gpurun): bash tools/gpu_session.sh   (AB_CONFIGS overrides the A/B list)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
ok() { case $1 in 0|1) return 0;; *) echo "stopping: rc=$1"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; ok $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; ok $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
rc=$?; echo "bench rc=$rc"; ok $rc
cat gpurun_out/bench1.json
timeout -k 10 300 python -u tools/ab_classify.py --rounds 3 --iters 3 --configs "${AB_CONFIGS:-3:1,4:1,5:1,6:1,7:1,20:1,21:1,22:1,9:1}" > gpurun_out/ab1.json 2> gpurun_out/ab1.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab1.json
