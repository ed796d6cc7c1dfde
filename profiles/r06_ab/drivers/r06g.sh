# r06g: round-end evidence of the round-6 build (2^26-slot tile launches, rings across calls, rows
# dealt): the GPU suite, bench + PMC (incl. the per-kernel HBM summary) + rocprof kernel stats, the
# lane-op reconciliation
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_round_end.sh r06g || exit 1
bash tools/gpu_lane_ops.sh r06g_lane_ops || exit 1
