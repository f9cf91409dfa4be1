# PMC passes over the conntrack walker (k_ct_walk) and the other CT kernels
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
OUT=gpurun_out/pmc_ct
mkdir -p $OUT
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS" "TCC_HIT_sum TCC_MISS_sum" "TA_BUSY_avr GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --kernel-include-regex "k_ct_" --output-format csv -d $OUT/p$i -o pmc -- python3 bench.py --config ct --steps 1 --warmup 0 --no-cpu-baseline --tuples 16777216 > $OUT/p$i.log 2>&1
  rc=$?; echo "pmc$i ($P) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
