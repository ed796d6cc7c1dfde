# r06r: evidence of the branch-free FP64 visit build (YK_NODE_BF=2, YK_STACK_EXACT=1 by default):
# the GPU suite (+ the shallow checked-stack test build), bench + PMC (per-kernel HBM) + rocprof
# kernel stats, the lane-op reconciliation, smoke, and the phase split (stamp builds) of the
# round-5 visit vs the branch-free one at 32 spp
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_round_end.sh r06r || exit 1
bash tools/gpu_lane_ops.sh r06r_lane_ops || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06r/smoke.log 2>&1 || { tail -20 gpurun_out/r06r/smoke.log; exit 1; }
tail -1 gpurun_out/r06r/smoke.log
bash tools/gpu_phases.sh 32 st_base st_bf2x > gpurun_out/r06r/phases.txt 2>&1 || { tail -20 gpurun_out/r06r/phases.txt; exit 1; }
cat gpurun_out/r06r/phases.txt
