set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/r5_m5; mkdir -p $OUT
for cfg in ctlb ct6 ctlb6 ct; do
CGPU_AB_CONFIG=$cfg timeout -k 10 300 python -u tools/diag_ab.py run product walk_w3 product walk_w3 > $OUT/ab_$cfg.log 2>&1; rc=$?; echo "ab $cfg rc=$rc"; grep variant $OUT/ab_$cfg.log; [ $rc -eq 0 ] || exit $rc
done
