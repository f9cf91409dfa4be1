set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/r5_k5; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ctlb6.py tests/test_gpu_ct6.py tests/test_gpu_ctlb.py > $OUT/pytest_ct.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_ct.log; [ $rc -eq 0 ] || exit $rc
CGPU_AB_CONFIG=ctlb6 timeout -k 10 300 python -u tools/diag_ab.py run head product svc_pre6_off head product > $OUT/ab_ctlb6.log 2>&1; rc=$?; echo "ab rc=$rc"; grep variant $OUT/ab_ctlb6.log; [ $rc -eq 0 ] || exit $rc
