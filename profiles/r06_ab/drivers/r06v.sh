# r06v: evidence of the build with slab pairs, scalar slot claims and 112-VGPR production render
# instances (counting instances under their own kernel name, uncapped): the GPU suite, bench + PMC
# + rocprof kernel stats, the lane-op reconciliation, smoke, and the phase split (stamp builds) of
# the branch-free visit build (r06r) vs this one at 32 spp
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_round_end.sh r06v || exit 1
bash tools/gpu_lane_ops.sh r06v_lane_ops || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06v/smoke.log 2>&1 || { tail -20 gpurun_out/r06v/smoke.log; exit 1; }
tail -1 gpurun_out/r06v/smoke.log
bash tools/gpu_phases.sh 32 st_bf2x st_new > gpurun_out/r06v/phases.txt 2>&1 || { tail -20 gpurun_out/r06v/phases.txt; exit 1; }
cat gpurun_out/r06v/phases.txt
