cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out &&
bash tools/gpu_round_end.sh r04i > gpurun_out/r04i.txt 2>&1
