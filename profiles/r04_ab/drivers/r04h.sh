cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04h &&
timeout -k 10 500 python tools/tile_ab.py base base@YKGPU_LAUNCH_SLOTS=67108864 base@YKGPU_FIRST_LAUNCH_OV=64 base@YKGPU_FIRST_LAUNCH_OV=128 base@YKGPU_LAUNCH_SLOTS=67108864@YKGPU_FIRST_LAUNCH_OV=128 > gpurun_out/r04h/tile8.txt 2>&1 &&
TILE=1920:512:2:0:cols timeout -k 10 300 python tools/tile_ab.py base base@YKGPU_FIRST_LAUNCH_OV=64 > gpurun_out/r04h/tile2.txt 2>&1 &&
TILE=1920:512:4:0:cols timeout -k 10 300 python tools/tile_ab.py base base@YKGPU_FIRST_LAUNCH_OV=64 base@YKGPU_LAUNCH_SLOTS=67108864 > gpurun_out/r04h/tile4.txt 2>&1
