# round-6 final bench lines (run on the GPU box from the repo root):
#   bash tools/r6_final_bench.sh <group>   -> gpurun_out/r6_final/bench_<name>.json
# groups: stateless, default, ct, ctlb, host, persist.  Each line under its own time limit; a
# failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/r6_final
mkdir -p $OUT
one() {  # name, limit, args...
  N=$1; T=$2; shift 2
  timeout -k 10 $T python -u bench.py "$@" > $OUT/bench_$N.json 2> $OUT/bench_$N.err
  rc=$?; echo "bench $N rc=$rc"; cut -c1-160 $OUT/bench_$N.json
  [ $rc -eq 0 ] || exit $rc
}
case $1 in
  stateless)
    one default 400
    for C in cascade pf6 v6 frames mapstate; do one $C 400 --config $C --steps 20 --warmup 3; done;;
  ct)
    one ct 500 --config ct --steps 20 --warmup 3
    one ct6 500 --config ct6 --steps 20 --warmup 3
    one ct_persist4 600 --config ct --steps 20 --warmup 3 --ct-persist 4
    one ct6_persist4 600 --config ct6 --steps 20 --warmup 3 --ct-persist 4;;
  ctlb)
    one ctlb 600 --config ctlb --steps 20 --warmup 3
    one ctlb6 600 --config ctlb6 --steps 20 --warmup 3;;
  host)
    for C in gpu frames cascade v6 pf6; do one ${C}hosttuples 400 --config $C --host-tuples --steps 5 --warmup 2 --no-cpu-baseline; done;;
  default)
    one default 400;;
  persist)
    one ct_persist4 600 --config ct --steps 20 --warmup 3 --ct-persist 4
    one ct6_persist4 600 --config ct6 --steps 20 --warmup 3 --ct-persist 4;;
esac
