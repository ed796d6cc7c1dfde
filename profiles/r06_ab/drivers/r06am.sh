# r06am: the N>1 rehearsal of the final build on one GPU (tools/gpu_multirank.sh: the contract's
# torchrun launch of bench.py at --gpus 2 and 8 over gloo, and the assembled-image check)
set -o pipefail
cd $GRAFT_REPO_ROOT
NS="2 8" bash tools/gpu_multirank.sh gpurun_out/r06am_multirank
