# rocprofv3 evidence for bench workloads (run on the GPU box from the repo root):
# per config, a kernel trace (--kernel-trace --stats) of the bench line and
# separate PMC passes over the same bench workload, summarized per step and
# stamped with the library identity (tools/pmc_summary.py).
#   bash tools/profile.sh <tag> <config> [<config> ...]   -> gpurun_out/prof_<tag>/<config>/
# Each step has its own time limit; a failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=$1
shift
W=1; K=2
for CONF in "$@"; do
  OUT=gpurun_out/prof_$TAG/$CONF
  mkdir -p $OUT
  # every config but pf6 runs one more step after the counter rebalance
  case $CONF in pf6) SKIP=$W;; *) SKIP=$((W + 1));; esac
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --config $CONF --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_under_rocprof.json 2> $OUT/bench.err
  rc=$?; echo "$CONF trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
  i=0
  for P in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $P --kernel-exclude-regex '__amd_rocclr_copyBuffer|__amd_rocclr_fillBuffer|at::native' --output-format csv -d $OUT/pmc$i -o pmc -- python3 bench.py --config $CONF --steps $K --warmup $W --no-parity > $OUT/pmc$i.log 2>&1
    rc=$?; echo "$CONF pmc$i ($P) rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python3 tools/pmc_summary.py $OUT $CONF $SKIP $K > $OUT/summary.log 2>&1 && echo "$CONF summary ok"
  find $OUT -name '*_counter_collection.csv' -size +20M -delete
done
