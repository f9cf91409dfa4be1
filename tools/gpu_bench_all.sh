# Bench every BASELINE config on one GPU (run on the gpurun box from the repo root):
#   bash tools/gpu_bench_all.sh [steps]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
S=${1:-10}
for C in gpu cascade pf6; do
  timeout -k 10 420 python -u bench.py --config $C --steps $S --warmup 3 > gpurun_out/bench_$C.json 2> gpurun_out/bench_$C.err
  rc=$?
  echo "bench $C rc=$rc"
  [ $rc -eq 0 ] || { tail -20 gpurun_out/bench_$C.err; exit $rc; }
  cat gpurun_out/bench_$C.json
done
