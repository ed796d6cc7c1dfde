# GPU parity tests of the current library, then A/B wall time against lib/abl variants.
# usage (on the GPU box): bash tools/gpu_ab.sh <spp> <variant> [<variant> ...]
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modes.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/ab_tests.log; exit 1; }
tail -2 gpurun_out/ab_tests.log
SPP=$1; shift
timeout -k 10 500 python -u tools/abtime.py $SPP base "$@" > gpurun_out/ab.log 2>&1 || { echo AB_FAILED; tail -30 gpurun_out/ab.log; exit 2; }
cat gpurun_out/ab.log
