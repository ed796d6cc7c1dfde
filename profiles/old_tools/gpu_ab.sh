# Parity of the current build (golden + BVH tests), then an A/B of library variants at one spp
# (tools/abtime.py) and the default bench.  usage: bash tools/gpu_ab.sh <tag> <spp> <variants...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; SPP=$2; shift 2
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$T/parity.log 2>&1 || { echo PARITY_FAILED; tail -30 gpurun_out/$T/parity.log; exit 1; }
tail -1 gpurun_out/$T/parity.log
timeout -k 10 900 python tools/abtime.py $SPP "$@" > gpurun_out/$T/ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab.txt; exit 2; }
cat gpurun_out/$T/ab.txt
timeout -k 10 400 python bench.py --no-cpu-baseline --no-modes > gpurun_out/$T/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/$T/bench.log; exit 3; }
grep '^{' gpurun_out/$T/bench.log | tail -1 | cut -c1-400
