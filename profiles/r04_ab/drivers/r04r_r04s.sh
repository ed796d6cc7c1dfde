cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04r &&
bash tools/gpu_bench_ab.sh r04r/bab base base@YKGPU_WARM_PER_CU=16 base@YKGPU_WARM_PER_CU=64 base@YKGPU_RED_BLOCKS=2 base@YKGPU_RED_BLOCKS=8 > gpurun_out/r04r/bench_ab.txt 2>&1 &&
mkdir -p gpurun_out/r04s &&
AB_REPS=4 timeout -k 10 600 python tools/abtime.py 512 base base@YKGPU_FIRST_LAUNCH=32 base@YKGPU_FIRST_LAUNCH=16@YKGPU_SCHED_GROW=2 > gpurun_out/r04s/ab_synced_first32.txt 2>&1 &&
YKGPU_FIRST_LAUNCH=32 YKGPU_TIMELINE=1 timeout -k 10 300 python tools/variance_probe.py 20 > gpurun_out/r04s/variance_first32.json 2> gpurun_out/r04s/variance_first32_timeline.txt
