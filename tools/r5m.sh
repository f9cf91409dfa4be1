set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/r5_m4; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ct.py tests/test_gpu_ct6.py tests/test_gpu_ctlb.py tests/test_gpu_ctlb6.py > $OUT/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
for cfg in ct ct6; do
CGPU_AB_CONFIG=$cfg timeout -k 10 300 python -u tools/diag_ab.py run product prep_q3 prep_q2 product prep_q3 prep_q2 > $OUT/ab_$cfg.log 2>&1; rc=$?; echo "ab $cfg rc=$rc"; grep variant $OUT/ab_$cfg.log; [ $rc -eq 0 ] || exit $rc
done
