# The whole GPU test suite, then an A/B of library variants (tools/abtime.py) at one spp.
# usage: bash tools/gpu_tests_ab.sh <tag> <spp> <variants...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; SPP=$2; shift 2
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
timeout -k 10 900 python tools/abtime.py $SPP "$@" > gpurun_out/$T/ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab.txt; exit 2; }
cat gpurun_out/$T/ab.txt
