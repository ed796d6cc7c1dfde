# r05af: round-end evidence of the build with the four-walk deferred warm-up as the default: the GPU
# suite, bench + PMC + rocprof kernel stats (tools/gpu_round_end.sh), the lane-op reconciliation
# against the new warm-up kernel (tools/gpu_lane_ops.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_round_end.sh r05af || exit 1
bash tools/gpu_lane_ops.sh r05af_lane_ops || exit 1
