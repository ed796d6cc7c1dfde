cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04g &&
timeout -k 10 500 python tools/tile_ab.py base base@YKGPU_WARM_RING=4 base@YKGPU_LAUNCH_SLOTS=16777216 base@YKGPU_LAUNCH_SLOTS=8388608 base@YKGPU_LAUNCH_SLOTS=8388608@YKGPU_WARM_RING=4 base@YKGPU_SCHED_GROW_OV=2 > gpurun_out/r04g/tile8.txt 2>&1 &&
TILE=1920:512:4:0:cols timeout -k 10 300 python tools/tile_ab.py base base@YKGPU_LAUNCH_SLOTS=8388608 base@YKGPU_WARM_RING=4 > gpurun_out/r04g/tile4.txt 2>&1 &&
TILE=1920:512:1:0:cols CALLS=4 timeout -k 10 400 python tools/tile_ab.py base base@YKGPU_WARM_RING=4 base@YKGPU_SCHED_GROW_OV=2 > gpurun_out/r04g/frame.txt 2>&1
