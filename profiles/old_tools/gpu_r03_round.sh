# Round-3 evidence of the current build on the GPU box: the whole -m gpu suite, then PMC passes +
# bench + rocprofv3 kernel trace (tools/gpu_profile_all.sh), then a kernel trace of configs 4 and 5
# (tools/configs45.py) for their per-launch unions.   usage: bash tools/gpu_r03_round.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r03i}
mkdir -p gpurun_out/$T
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
bash tools/gpu_profile_all.sh $T || exit 2
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/kt45 -o run -- python3 tools/configs45.py c4 c5 > gpurun_out/$T/kt45.log 2>&1 || { echo KT45_FAILED; tail -20 gpurun_out/$T/kt45.log; exit 3; }
grep -E "^c[45]:" gpurun_out/$T/kt45.log
