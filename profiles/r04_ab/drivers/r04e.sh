cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
bash tools/gpu_round_end.sh r04e > gpurun_out/r04e.txt 2>&1 &&
NS="2 8" bash tools/gpu_multirank.sh gpurun_out/r04e_multirank >> gpurun_out/r04e.txt 2>&1
