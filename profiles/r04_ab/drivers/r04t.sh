cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04t &&
timeout -k 10 300 python tools/tile_timeline.py 1920 512 8 0 cols 4 > gpurun_out/r04t/tile_tl.json 2> gpurun_out/r04t/tile_tl.txt &&
timeout -k 10 400 python tools/tile_ab.py base base@YKGPU_WARM_RING=4 base@YKGPU_COL_RING=3 base@YKGPU_WARM_RING=2 > gpurun_out/r04t/tile8.txt 2>&1
