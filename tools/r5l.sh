set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/r5_l3; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_frames.py > $OUT/pytest_frames.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest_frames.log; [ $rc -eq 0 ] || exit $rc
CGPU_AB_CONFIG=frames CGPU_AB_REBALANCE=1 timeout -k 10 300 python -u tools/diag_ab.py run product ff_pool0 ff_pool8 ff_pool2 product ff_pool0 ff_pool8 ff_pool2 > $OUT/ab_frames_pool.log 2>&1; rc=$?; echo "ab rc=$rc"; grep variant $OUT/ab_frames_pool.log; [ $rc -eq 0 ] || exit $rc
