set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/r5_k3; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_ctlb.py tests/test_gpu_ctlb6.py tests/test_gpu_ct.py > $OUT/pytest_ct.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_ct.log; [ $rc -eq 0 ] || exit $rc
for cfg in ctlb; do
CGPU_AB_CONFIG=$cfg timeout -k 10 300 python -u tools/diag_ab.py run head product walk_svc_minb3 head product walk_svc_minb3 > $OUT/ab_$cfg.log 2>&1; rc=$?; echo "ab $cfg rc=$rc"; grep variant $OUT/ab_$cfg.log; [ $rc -eq 0 ] || exit $rc
done
