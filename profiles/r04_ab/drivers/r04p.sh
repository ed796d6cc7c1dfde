cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04p &&
bash tools/gpu_bench_ab.sh r04p/bab base base@YKGPU_LAUNCH_SPP=24 base@YKGPU_LAUNCH_SPP=40 > gpurun_out/r04p/bench_ab.txt 2>&1 &&
AB_PREC=1 timeout -k 10 600 python tools/abtime.py 512 base base@YKGPU_WARM_PER_CU=4 base@YKGPU_WARM_PER_CU=8 > gpurun_out/r04p/ab_f32_warm.txt 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_tiles_rccl.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r04p/rccl_test.log 2>&1
