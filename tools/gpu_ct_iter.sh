# conntrack iteration: parity tests, then the full bench + kernel trace
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
stop() { echo "stopping: $1 rc=$2"; exit $2; }
timeout -k 10 400 python -u -m pytest tests/test_gpu_ct.py -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_ct.log 2>&1
rc=$?; echo "ct pytest rc=$rc"; tail -15 gpurun_out/pytest_ct.log; [ $rc = 0 ] || stop ct $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ct -o run -- python3 bench.py --config ct --steps 5 --warmup 2 > gpurun_out/bench_ct.json 2> gpurun_out/bench_ct.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_ct.json; [ $rc = 0 ] || stop bench $rc
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open('gpurun_out/prof_ct/run_kernel_stats.csv')))[:8]:
    print(r['Name'][:60], r['Calls'], r['AverageNs'], r['Percentage'])
PY
