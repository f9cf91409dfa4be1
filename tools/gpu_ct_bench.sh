# conntrack bench: a small run, the full config, and the
# rocprof kernel trace of the full config.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
stop() { echo "stopping: $1 rc=$2"; exit $2; }
timeout -k 10 300 python -u bench.py --config ct --tuples 4000000 --steps 3 --warmup 1 > gpurun_out/bench_ct_small.json 2> gpurun_out/bench_ct_small.err
rc=$?; echo "small rc=$rc"; cat gpurun_out/bench_ct_small.json; tail -3 gpurun_out/bench_ct_small.err; [ $rc = 0 ] || stop small $rc
timeout -k 10 600 python -u bench.py --config ct --steps 5 --warmup 2 > gpurun_out/bench_ct.json 2> gpurun_out/bench_ct.err
rc=$?; echo "full rc=$rc"; cat gpurun_out/bench_ct.json; tail -3 gpurun_out/bench_ct.err; [ $rc = 0 ] || stop full $rc
if [ "${1:-}" = "prof" ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ct -o run -- python3 bench.py --config ct --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/prof_ct_bench.json 2> gpurun_out/prof_ct_bench.err
rc=$?; echo "prof rc=$rc"; [ $rc = 0 ] || stop prof $rc
fi
