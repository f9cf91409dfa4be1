set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/r5_m; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_frames.py tests/test_gpu_ct.py tests/test_gpu_lb.py > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in gpu frames ct; do
CGPU_AB_CONFIG=$cfg CGPU_AB_REBALANCE=1 timeout -k 10 300 python -u tools/diag_ab.py run product pk_copies1 product pk_copies1 > $OUT/ab_$cfg.log 2>&1; rc=$?; echo "ab $cfg rc=$rc"; grep variant $OUT/ab_$cfg.log; [ $rc -eq 0 ] || exit $rc
done
