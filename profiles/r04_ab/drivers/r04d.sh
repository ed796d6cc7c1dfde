cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04d &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04d/gpu_tests.log 2>&1 &&
AB_PREC=1 timeout -k 10 600 python tools/abtime.py 512 base fold0 pairs > gpurun_out/r04d/ab_f32.txt 2>&1 &&
timeout -k 10 600 python tools/abtime.py 512 base k16 k16@YKGPU_COL_RING=2 > gpurun_out/r04d/ab_k16.txt 2>&1 &&
AB_W=3840 AB_ROWS=0:270:8 timeout -k 10 600 python tools/abtime.py 1024 base base@YKGPU_COL_RING=2 k16 k16@YKGPU_COL_RING=2 > gpurun_out/r04d/ab_c4tile.txt 2>&1 &&
bash tools/gpu_bench_ab.sh r04d/bab base base@YKGPU_COL_RING=2 base@YKGPU_COL_RING=3 sched8 > gpurun_out/r04d/bench_ab.txt 2>&1 &&
YKGPU_TIMELINE=1 timeout -k 10 300 python tools/variance_probe.py 20 > gpurun_out/r04d/variance.json 2> gpurun_out/r04d/variance_timeline.txt &&
timeout -k 10 400 python bench.py --no-cpu-baseline --no-modes --no-configs > gpurun_out/r04d/bench_tiles.log 2>&1
