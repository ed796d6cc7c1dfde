set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_modes.py tests/test_gpu_parity.py tests/test_cli.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_tests2.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests2.log; exit 1; }
tail -3 gpurun_out/gpu_tests2.log
timeout -k 10 300 python -u tools/modes_time.py 512 16 > gpurun_out/modes.log 2>&1 || { echo MODES_FAILED; tail -30 gpurun_out/modes.log; exit 2; }
cat gpurun_out/modes.log
