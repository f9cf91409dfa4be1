# copy the judged parts of a tools/profile.sh run into profiles/:
#   bash tools/keep_profile.sh <tag> <config>...  -> profiles/<tag>_prof/<config>/, profiles/traffic_<config>.json
set -e
TAG=$1; shift
for C in "$@"; do
  S=gpurun_out/prof_$TAG/$C; D=profiles/${TAG}_prof/$C
  mkdir -p $D
  cp $S/bench_under_rocprof.json $S/pmc_summary.json $S/summary.log $S/traffic.json $D/
  cp $S/trace/run_kernel_stats.csv $D/kernel_stats.csv
  cp $S/traffic.json profiles/traffic_$C.json
done
