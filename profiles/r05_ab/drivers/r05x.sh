# r05x: the deferred-lens warm-up at 24 VGPRs (five warm-up waves per SIMD beside the render's
# three; 32 VGPRs of spills) against base (32 VGPRs, four waves): bench steps, 3 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05x
mkdir -p gpurun_out/$T
for rnd in 0 1 2; do
  for v in base d24; do
    if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
    YKGPU_LIB_OVERRIDE=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes --no-configs --no-tiles > gpurun_out/$T/bench_${v}_$rnd.log 2>&1 || { echo BENCH_FAILED $v; tail -5 gpurun_out/$T/bench_${v}_$rnd.log; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/$T/bench_${v}_$rnd.log') if l.startswith('{')][-1])
print($rnd, '$v', d['value'], d['ms_per_step'])"
  done
done
