# PMC passes over several classify configurations (diagnostics).
# usage: PMC_CONFIGS="13:25 14:25 14:12" bash tools/pmc_ab.sh   (VARIANT:LOADPCT)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for C in ${PMC_CONFIGS}; do
  V=${C%%:*}; P=${C##*:}
  OUT=gpurun_out/pmcab_${V}_${P}
  mkdir -p $OUT
  i=0
  for PASS in "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" "TA_BUSY_avr GRBM_GUI_ACTIVE" "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES"; do
    i=$((i+1))
    CGPU_CLASSIFY_VARIANT=$V CGPU_POL_LOAD_PCT=$P timeout -s KILL 120 rocprofv3 --pmc $PASS --kernel-include-regex k_classify --output-format csv -d $OUT/pmc$i -o pmc -- python3 tools/pmc_driver.py > $OUT/pmc$i.log 2>&1
    rc=$?; echo "$C pmc$i rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/pmc_summary.py $OUT > /dev/null && python3 -c "import json;d=json.load(open('$OUT/pmc_summary.json'));print('$C', d['meta'].get('kernel','')[:60], json.dumps({k:round(v) for k,v in d['counters'].items()}))"
done
