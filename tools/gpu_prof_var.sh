# rocprofv3 kernel stats of one A/B configuration list (diagnostics)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_classify.py --rounds 3 --iters 3 --configs "${AB_CONFIGS}" > gpurun_out/ab3.json 2> gpurun_out/ab3.err
rc=$?; echo "ab rc=$rc"; cat gpurun_out/ab3.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pv -o run -- python3 tools/ab_classify.py --rounds 1 --iters 3 --configs "${AB_CONFIGS}" > gpurun_out/pv.log 2>&1
rc=$?; echo "prof rc=$rc"; find gpurun_out/pv -name "*kernel_stats.csv" -exec cat {} \;
