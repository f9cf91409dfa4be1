# Bench line of every workload, then the config-2 rocprof trace + PMC passes
# (run on the GPU box from the repo root via gpurun):
#   bash tools/gpu_configs.sh <tag> [configs...]  -> gpurun_out/<tag>/bench_<config>.{json,err}
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-cfg}
shift
CONFIGS=${@:-gpu cascade pf6 v6 frames ct mapstate}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for C in $CONFIGS; do
  timeout -k 10 400 python -u bench.py --config $C --steps 20 --warmup 3 > $OUT/bench_$C.json 2> $OUT/bench_$C.err
  rc=$?; echo "bench $C rc=$rc"; cat $OUT/bench_$C.json
  [ $rc -eq 0 ] || exit $rc
done
