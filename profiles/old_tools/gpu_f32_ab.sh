cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r02am
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/r02am/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r02am/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r02am/gpu_tests.log
AB_PREC=1 timeout -k 10 600 python tools/abtime.py 512 base head > gpurun_out/r02am/ab_f32.txt 2>&1 || exit 2
cat gpurun_out/r02am/ab_f32.txt
