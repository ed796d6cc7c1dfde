cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04j &&
bash tools/gpu_phases.sh 32 stamps > gpurun_out/r04j/phases_32spp.txt 2>&1
