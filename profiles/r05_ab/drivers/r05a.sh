# r05a: GPU suite at the round-5 start build (dual kernel out, A/B knobs gated, exact ring
# geometry, memory-aware launch sizing, lane-op counters), the new ubench ops, one bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05a
mkdir -p gpurun_out/$T
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$T/gpu_tests.log
timeout -k 10 300 tools/ubench gpurun_out/$T/ubench.jsonl > gpurun_out/$T/ubench.txt 2>&1 || { echo UBENCH_FAILED; tail -5 gpurun_out/$T/ubench.txt; exit 1; }
timeout -k 10 500 python bench.py > gpurun_out/$T/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/$T/bench.log; exit 1; }
grep '^{' gpurun_out/$T/bench.log | tail -1 > gpurun_out/$T/bench.json
python3 -c "import json; b=json.load(open('gpurun_out/$T/bench.json')); print(b['value'], b['ms_per_step'], b['roofline']['frac'])"
