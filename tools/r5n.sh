set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/r5_n; mkdir -p $OUT
for cfg in ct ct6; do
CGPU_AB_CONFIG=$cfg timeout -k 10 300 python -u tools/diag_ab.py run product ret_default ct_noret product ret_default ct_noret > $OUT/ab_$cfg.log 2>&1; rc=$?; echo "ab $cfg rc=$rc"; grep variant $OUT/ab_$cfg.log; [ $rc -eq 0 ] || exit $rc
done
