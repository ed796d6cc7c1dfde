cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04r &&
bash tools/gpu_bench_ab.sh r04r/bab base base@YKGPU_WARM_PER_CU=16 base@YKGPU_WARM_PER_CU=64 base@YKGPU_RED_BLOCKS=2 base@YKGPU_RED_BLOCKS=8 > gpurun_out/r04r/bench_ab.txt 2>&1
