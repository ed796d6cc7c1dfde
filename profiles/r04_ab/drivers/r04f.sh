cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04f &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04f/gpu_tests.log 2>&1 &&
timeout -k 10 300 python tools/tile_timeline.py 1920 512 8 0 cols 4 > gpurun_out/r04f/tile_tl.json 2> gpurun_out/r04f/tile_tl.txt &&
YKGPU_FIRST_LAUNCH_OV=32 timeout -k 10 300 python tools/tile_timeline.py 1920 512 8 0 cols 4 > gpurun_out/r04f/tile_tl_ov32.json 2> gpurun_out/r04f/tile_tl_ov32.txt &&
timeout -k 10 300 python tools/tile_timeline.py 1920 512 1 0 cols 4 > gpurun_out/r04f/frame_tl.json 2> gpurun_out/r04f/frame_tl.txt &&
bash tools/gpu_bench_ab.sh r04f/bab base base@YKGPU_FIRST_LAUNCH_OV=4@YKGPU_SCHED_GROW_OV=2 base@YKGPU_FIRST_LAUNCH_OV=32 base@YKGPU_LAUNCH_SPP=48 base@YKGPU_LAUNCH_SPP=64 > gpurun_out/r04f/bench_ab.txt 2>&1 &&
AB_PREC=1 timeout -k 10 600 python tools/abtime.py 512 base nopairs32 > gpurun_out/r04f/ab_f32.txt 2>&1
