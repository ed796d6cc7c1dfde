# r05al: the render's refill reads only the StartRec (empty slots marked in it, kPadSlot; the
# processing order and the seed read only for a start the render makes itself; the scratch engine
# recovers the seed from its cursor): the GPU suite on the new build (base), then synced calls with
# image hashes and bench steps (3 rounds) against head (the build before it).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05al
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$T/gpu_tests.log
AB_REPS=2 timeout -k 10 300 python tools/abtime.py 512 base head > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
for rnd in 0 1 2; do
  for v in base head; do
    if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
    YKGPU_LIB_OVERRIDE=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes --no-configs --no-tiles > gpurun_out/$T/bench_${v}_$rnd.log 2>&1 || { echo BENCH_FAILED $v; tail -5 gpurun_out/$T/bench_${v}_$rnd.log; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/$T/bench_${v}_$rnd.log') if l.startswith('{')][-1])
print($rnd, '$v', d['value'], d['ms_per_step'])"
  done
done
