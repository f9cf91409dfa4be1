set -e
mkdir -p gpurun_out/r6_j
for c in cascade v6 pf6 gpu; do
  timeout -k 10 300 python -u bench.py --config $c --host-tuples --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r6_j/host_$c.json 2> gpurun_out/r6_j/host_$c.err
done
