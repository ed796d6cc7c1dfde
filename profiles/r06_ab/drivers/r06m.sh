# r06m: round-end evidence of the final tree (122 GPU tests): the GPU suite, bench + PMC (per-kernel
# HBM) + rocprof kernel stats, the lane-op reconciliation, smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_round_end.sh r06m || exit 1
bash tools/gpu_lane_ops.sh r06m_lane_ops || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06m/smoke.log 2>&1 || { tail -20 gpurun_out/r06m/smoke.log; exit 1; }
tail -1 gpurun_out/r06m/smoke.log
