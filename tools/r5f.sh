set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/r5_f; mkdir -p $OUT
CT_SCAN_DIAG=1 timeout -k 10 300 python -u tools/ct_scan.py 32 > $OUT/ct_scan.log 2>&1; rc=$?; echo "ct_scan rc=$rc"; tail -4 $OUT/ct_scan.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_ct -o run -- python3 bench.py --config ct --steps 5 --warmup 2 --no-parity > $OUT/trace_ct.json 2> $OUT/trace_ct.err; rc=$?; echo "trace ct rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/host_ab.py tuples product hs_g256 hs_g512 hs_g64 hs_chunk23 hs_chunk21 product > $OUT/host_ab.log 2>&1; rc=$?; echo "host_ab rc=$rc"; cat $OUT/host_ab.log | grep variant
