# r05b: lane-op reconciliation probe (8 spp of the headline frame), then the full evidence run
# (PMC passes, bench line, rocprofv3 kernel trace) of the same build.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/gpu_lane_ops.sh r05b 8 > gpurun_out/r05b_lane_ops.log 2>&1 || { echo LANE_OPS_FAILED; tail -30 gpurun_out/r05b_lane_ops.log; exit 1; }
tail -45 gpurun_out/r05b_lane_ops.log
bash tools/gpu_profile_all.sh r05b || exit 1
