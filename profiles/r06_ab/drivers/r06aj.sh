# r06aj: round-end evidence of the near-clamp build — lane-op reconciliation first (installed as
# profiles/pmc_lane_ops.json so the bench line quotes this build's counters), then the whole -m gpu
# suite, PMC passes, bench, kernel trace (tools/gpu_round_end.sh)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_lane_ops.sh r06aj_lane_ops || exit 1
cp gpurun_out/r06aj_lane_ops/pmc_lane_ops.json profiles/pmc_lane_ops.json
bash tools/gpu_round_end.sh r06aj
