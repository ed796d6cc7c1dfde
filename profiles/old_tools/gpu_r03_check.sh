# Whole GPU suite, the default bench line (configs 4/5 included) and the N = 2, 3, 8 torchrun
# rehearsal on one GPU (gloo ranks sharing it).  usage: bash tools/gpu_r03_check.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r03c}
mkdir -p gpurun_out/$T
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -1 gpurun_out/$T/gpu_tests.log
S=$(date +%s)
timeout -k 10 400 python bench.py > gpurun_out/$T/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/$T/bench.log; exit 2; }
echo "bench wall $(( $(date +%s) - S )) s"
grep '^{' gpurun_out/$T/bench.log | tail -1 > gpurun_out/$T/bench.json
python3 -c "
import json; d=json.load(open('gpurun_out/$T/bench.json'))
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('parity_vs_cpu'))
for k,v in d.get('configs',{}).items(): print(k, v['value'], v['ms'], v['roofline']['frac'], v['parity_vs_cpu'], v['device_bytes'])
"
bash tools/gpu_multirank.sh gpurun_out/$T/multirank || exit 3
cat gpurun_out/$T/multirank/check_n*.log | grep world
