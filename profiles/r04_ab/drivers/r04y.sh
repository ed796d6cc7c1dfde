cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04y &&
for rep in 0 1; do for v in "YKGPU_LAUNCH_SPP=32" "YKGPU_LAUNCH_SPP=64" "YKGPU_LAUNCH_SPP=121" "YKGPU_WARM_RING=2"; do env $v timeout -k 10 300 python tools/configs45.py c5 2>&1 | grep -v amdgpu | sed "s/^/$rep $v /"; done; done > gpurun_out/r04y/c5_rule.txt
