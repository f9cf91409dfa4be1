# config 5: cascade bench per VIP-bitmap size (bits per frontend)
#   LB_VIP_BITS="8 16 32" bash tools/gpu_lb_ab.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
for B in ${LB_VIP_BITS:-8 16 32}; do
  CGPU_LB_VIP_BITS=$B timeout -k 10 400 python -u bench.py --config cascade --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_cascade_b$B.json 2> gpurun_out/bench_cascade_b$B.err
  rc=$?; echo "bits=$B rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/bench_cascade_b$B.err; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/bench_cascade_b$B.json')); print('bits=$B', d['value'], d['config']['kernel_ms'], d['config']['parity_vs_oracle'])"
done
