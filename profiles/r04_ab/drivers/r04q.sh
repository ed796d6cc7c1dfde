cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04q &&
bash tools/gpu_bench_ab.sh r04q/bab base base@YKGPU_LAUNCH_SPP=36 base@YKGPU_LAUNCH_SPP=40 base@YKGPU_LAUNCH_SPP=44 > gpurun_out/r04q/bench_ab.txt 2>&1 &&
bash tools/gpu_bench_ab.sh r04q/bab2 base base@YKGPU_LAUNCH_SPP=40 > gpurun_out/r04q/bench_ab2.txt 2>&1
