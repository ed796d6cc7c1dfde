# GPU tests, the N>1 rehearsal and the default bench of the current build.
# usage: bash tools/gpu_r02b.sh <tag>   → gpurun_out/<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r02b}
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$T/gpu_tests.log
bash tools/gpu_multirank.sh gpurun_out/$T/multirank || exit 2
timeout -k 10 400 python bench.py > gpurun_out/$T/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/$T/bench.log; exit 3; }
grep '^{' gpurun_out/$T/bench.log | tail -1 > gpurun_out/$T/bench.json
cat gpurun_out/$T/bench.json
