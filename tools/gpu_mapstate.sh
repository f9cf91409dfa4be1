set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_l3.py -x -q --timeout 180 --timeout-method thread > gpurun_out/pytest_l3.log 2>&1
rc=$?; echo "l3 pytest rc=$rc"; tail -3 gpurun_out/pytest_l3.log; [ $rc = 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_l3 -o run -- python3 bench.py --config mapstate --steps 5 --warmup 1 > gpurun_out/bench_mapstate.json 2> gpurun_out/bench_mapstate.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_mapstate.json; tail -2 gpurun_out/bench_mapstate.err; [ $rc = 0 ] || exit $rc
python3 - <<'PY'
import csv
for r in list(csv.DictReader(open('gpurun_out/prof_l3/run_kernel_stats.csv')))[:5]:
    print(r['Name'][:60], r['Calls'], r['AverageNs'], r['Percentage'])
PY
