# rocprofv3 kernel traces (stats) of bench workloads, one after another:
#   bash tools/gpu_trace.sh <tag> <config[:extra args]> ...  -> gpurun_out/<tag>/<config>/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=$1; shift
for C in "$@"; do
  NAME=${C%%:*}; EXTRA=${C#*:}; [ "$EXTRA" = "$C" ] && EXTRA=""
  OUT=gpurun_out/$TAG/$NAME$(echo "$EXTRA" | tr -d ' -')
  mkdir -p $OUT
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --config $NAME --steps 5 --warmup 2 --no-cpu-baseline $EXTRA > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; echo "trace $C rc=$rc"; cut -c1-200 $OUT/bench.json
  [ $rc -eq 0 ] || exit $rc
done
