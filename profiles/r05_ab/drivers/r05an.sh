# r05an: the FP32 render's starts read the StartRecF alone too (as r05al for FP64): the GPU suite on
# the new build (base), then synced FP32 calls (AB_PREC=1) with image hashes against head (the build
# before it, same two-unit build), and the bench's FP32 mode line, 2 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05an
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$T/gpu_tests.log
AB_PREC=1 AB_REPS=2 timeout -k 10 300 python tools/abtime.py 512 base head > gpurun_out/$T/ab512_fp32.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512_fp32.txt; exit 1; }
cat gpurun_out/$T/ab512_fp32.txt
for rnd in 0 1; do
  for v in base head; do
    if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
    YKGPU_LIB_OVERRIDE=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-configs --no-tiles > gpurun_out/$T/bench_${v}_$rnd.log 2>&1 || { echo BENCH_FAILED $v; tail -5 gpurun_out/$T/bench_${v}_$rnd.log; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/$T/bench_${v}_$rnd.log') if l.startswith('{')][-1])
print($rnd, '$v', d['value'], d['ms_per_step'], {k: v['value'] for k, v in d['modes'].items()})"
  done
done
