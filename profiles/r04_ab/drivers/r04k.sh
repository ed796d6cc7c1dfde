cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04k &&
bash tools/gpu_bench_ab.sh r04k/bab base base@YKGPU_ORDER=1 > gpurun_out/r04k/bench_ab.txt 2>&1 &&
timeout -k 10 300 python tools/tile_ab.py base base@YKGPU_ORDER=1 > gpurun_out/r04k/tile8.txt 2>&1 &&
timeout -k 10 300 python tools/abtime.py 512 base base@YKGPU_ORDER=1 > gpurun_out/r04k/ab_synced.txt 2>&1
