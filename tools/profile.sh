# rocprofv3 passes for the bench workload (run on the GPU box from the repo root)
# usage: bash tools/profile.sh <tag> [config] [kernel-regex]   -> gpurun_out/prof_<tag>/
#   config: gpu (default) / cascade / pf6; kernel-regex: k_classify (default)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-r1}
CONF=${2:-gpu}
KRE=${3:-k_classify}
export CGPU_PMC_CONFIG=$CONF
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --config $CONF --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_sum" "TA_BUSY_avr GRBM_GUI_ACTIVE" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU" "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_WR" "TCC_EA0_ATOMIC_sum"; do
  i=$((i+1))
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex $KRE --output-format csv -d $OUT/pmc$i -o pmc -- python3 tools/pmc_driver.py > $OUT/pmc$i.log 2>&1
  rc=$?; echo "pmc$i ($P) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py $OUT $KRE $CONF > /dev/null && echo summary ok
