# the conntrack workloads: profile, install the stamped traffic in this
# (scratch) tree, then their bench lines
set -o pipefail
cd "$GRAFT_REPO_ROOT"
bash tools/profile.sh r4d ct ct6 ctlb ctlb6 || exit $?
for C in ct ct6 ctlb ctlb6; do cp gpurun_out/prof_r4d/$C/traffic.json profiles/traffic_$C.json || exit 1; done
bash tools/gpu_quick.sh r4_final4 "" "ct ct6 ctlb ctlb6"
