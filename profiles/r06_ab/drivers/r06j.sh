# r06j: round-end evidence of the final round-6 build: the GPU suite, bench + PMC (per-kernel HBM) +
# rocprof kernel stats, the lane-op reconciliation, smoke, and the N = 2, 8 rehearsal (torchrun,
# gloo ranks on one GPU, rows dealt)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_round_end.sh r06j || exit 1
bash tools/gpu_lane_ops.sh r06j_lane_ops || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06j/smoke.log 2>&1 || { tail -20 gpurun_out/r06j/smoke.log; exit 1; }
NS="2 8" bash tools/gpu_multirank.sh gpurun_out/r06j_multirank || exit 1
