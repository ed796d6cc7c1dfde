# r05av: round-end evidence of the final build (four-walk warm-up, StartRec-only starts, unwind shared with the reduce): the GPU
# suite, bench + PMC + rocprof kernel stats (tools/gpu_round_end.sh), the lane-op reconciliation
# against the new warm-up kernel (tools/gpu_lane_ops.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_round_end.sh r05av || exit 1
bash tools/gpu_lane_ops.sh r05av_lane_ops || exit 1
