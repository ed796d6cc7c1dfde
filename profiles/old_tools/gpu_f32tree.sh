# FP32 tree check on the GPU box: the modes tests, then the per-mode timing of the headline workload.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_modes.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/f32_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/f32_tests.log; exit 1; }
tail -3 gpurun_out/f32_tests.log
timeout -k 10 300 python -u tools/modes_time.py 512 512 > gpurun_out/modes.log 2>&1 || { echo MODES_FAILED; tail -30 gpurun_out/modes.log; exit 2; }
cat gpurun_out/modes.log
