# r05ao: round-end evidence of the final build (four-walk warm-up, StartRec-only starts): the GPU
# suite, bench + PMC + rocprof kernel stats (tools/gpu_round_end.sh), the lane-op reconciliation
# against the new warm-up kernel (tools/gpu_lane_ops.sh).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_round_end.sh r05ao || exit 1
bash tools/gpu_lane_ops.sh r05ao_lane_ops || exit 1
