cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out/r04c &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04c/gpu_tests.log 2>&1 &&
bash tools/gpu_bench_ab.sh r04c/bab base base@YKGPU_OVERLAP=0 > gpurun_out/r04c/bench_ab.txt 2>&1 &&
timeout -k 10 600 python tools/variance_ab.py 20 base base@YKGPU_SCHED_GROW=2 base@YKGPU_FIRST_LAUNCH=4@YKGPU_SCHED_GROW=2 base@YKGPU_FIRST_LAUNCH=16@YKGPU_SCHED_GROW=2 > gpurun_out/r04c/variance_ab.txt 2>&1 &&
YKGPU_DUAL=0 bash tools/pmc_profile.sh gpurun_out/r04c/pmc_single > gpurun_out/r04c/pmc_single.log 2>&1 &&
YKGPU_DUAL=1 bash tools/pmc_profile.sh gpurun_out/r04c/pmc_dual > gpurun_out/r04c/pmc_dual.log 2>&1 ;
timeout -k 10 120 rocprofv3 -L > gpurun_out/r04c/counters.txt 2>&1
