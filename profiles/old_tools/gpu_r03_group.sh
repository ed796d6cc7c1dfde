# Multi-device group tests + the chip-level VALU rates (ubench) on the GPU box.
# usage: bash tools/gpu_r03_group.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r03b}
mkdir -p gpurun_out/$T
timeout -k 10 300 python -u -m pytest tests/test_gpu_group.py tests/test_abi.py -m "gpu or not gpu" -x -v --timeout 120 --timeout-method thread > gpurun_out/$T/group_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/$T/group_tests.log; exit 1; }
tail -3 gpurun_out/$T/group_tests.log
timeout -k 10 240 tools/ubench gpurun_out/$T/ubench.jsonl > gpurun_out/$T/ubench.txt 2>&1 || { echo UBENCH_FAILED; tail -5 gpurun_out/$T/ubench.txt; exit 2; }
grep chip gpurun_out/$T/ubench.txt
