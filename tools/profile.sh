# rocprofv3 passes for the bench workload (run on the GPU box from the repo root)
# usage: bash tools/profile.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=${1:-r1}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
find $OUT/trace -name "*stats*" | head
