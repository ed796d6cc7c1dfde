cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04x &&
for rep in 0 1; do for v in 32 64 128; do YKGPU_LAUNCH_SPP=$v timeout -k 10 300 python tools/configs45.py c5 2>&1 | grep -v amdgpu | sed "s/^/$rep spp$v /"; done; done > gpurun_out/r04x/c5_launch_spp.txt
