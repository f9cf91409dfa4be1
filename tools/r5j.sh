set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
OUT=gpurun_out/r5_j; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_frames.py > $OUT/pytest_frames.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_frames.log; [ $rc -eq 0 ] || exit $rc
CGPU_AB_CONFIG=frames CGPU_AB_SCHED=8 timeout -k 10 300 python -u tools/diag_ab.py run product ff_nostage ff_h1 product > $OUT/ab_frames_fused.log 2>&1; rc=$?; echo "ab fused rc=$rc"; grep variant $OUT/ab_frames_fused.log; [ $rc -eq 0 ] || exit $rc
CGPU_AB_CONFIG=frames CGPU_AB_SCHED=0 timeout -k 10 300 python -u tools/diag_ab.py run product product > $OUT/ab_frames_split.log 2>&1; rc=$?; echo "ab split rc=$rc"; grep variant $OUT/ab_frames_split.log; [ $rc -eq 0 ] || exit $rc
