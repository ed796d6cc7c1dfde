# r05ba: round-end evidence of the final build after the shared unwind was reverted (the r05ao code): the GPU
# suite, bench + PMC + rocprof kernel stats (tools/gpu_round_end.sh), the lane-op reconciliation
# against the new warm-up kernel (tools/gpu_lane_ops.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_round_end.sh r05ba || exit 1
bash tools/gpu_lane_ops.sh r05ba_lane_ops || exit 1
