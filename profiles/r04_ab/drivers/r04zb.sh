cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04zb &&
TILE=1920:512:2:0:cols timeout -k 10 400 python tools/tile_ab.py base base@YKGPU_LAUNCH_SLOTS=67108864 > gpurun_out/r04zb/tile2.txt 2>&1 &&
TILE=1920:512:4:0:cols timeout -k 10 400 python tools/tile_ab.py base base@YKGPU_LAUNCH_SLOTS=67108864 > gpurun_out/r04zb/tile4.txt 2>&1
