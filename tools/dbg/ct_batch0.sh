cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/dbg/ct_batch0.py 2>&1 | grep -v amdgpu.ids
CGPU_CT_SORT_BITS=32 timeout -k 10 200 python -u tools/dbg/ct_batch0.py 2>&1 | grep -v amdgpu.ids
