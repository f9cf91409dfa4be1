# v6 prefilter: GPU tests, then config-3 bench per packets-per-lane variant
# (run on the gpurun box from the repo root): bash tools/gpu_pf6_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread -k "prefilter" > gpurun_out/pytest_pf6.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_pf6.log; [ $rc -eq 0 ] || exit $rc
for Q in ${PF6_QS:-4 2 1}; do
  CGPU_PF6_Q=$Q timeout -k 10 400 python -u bench.py --config pf6 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_pf6_q${Q/:/w}.json 2> gpurun_out/bench_pf6_q${Q/:/w}.err
  rc=$?; echo "Q=$Q rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_pf6_q${Q/:/w}.err; exit $rc; }
  python -c "import json,sys; d=json.load(open('gpurun_out/bench_pf6_q${Q/:/w}.json')); print('Q=$Q', d['value'], d['config']['kernel_ms'], d['roofline']['frac'], d['config']['parity_vs_oracle'])"
done
