# r05t: lens deferral v2 with the ring sized to the launch (6 sigma over the rejections of a wave's
# slots): bench steps (3 interleaved rounds), then bench.py with configs 4 and 5 (config 5's
# 121-spp launches: 1640 rejections per wave) for base and ld2; the GPU suite on ld2.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05t
mkdir -p gpurun_out/$T
for rnd in 0 1 2; do
  for v in base ld2; do
    if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
    YKGPU_LIB_OVERRIDE=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes --no-configs --no-tiles > gpurun_out/$T/bench_${v}_$rnd.log 2>&1 || { echo BENCH_FAILED $v; tail -5 gpurun_out/$T/bench_${v}_$rnd.log; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/$T/bench_${v}_$rnd.log') if l.startswith('{')][-1])
print($rnd, '$v', d['value'], d['ms_per_step'], 'call_gb', round(d['roofline']['hbm']['call_bytes']/1e9,2))"
  done
done
for v in base ld2; do
  if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
  YKGPU_LIB_OVERRIDE=$L timeout -k 10 400 python bench.py --no-cpu-baseline --no-modes --no-tiles --steps 2 --warmup 1 > gpurun_out/$T/cfg_$v.log 2>&1 || { echo CFG_FAILED $v; tail -5 gpurun_out/$T/cfg_$v.log; exit 1; }
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/$T/cfg_$v.log') if l.startswith('{')][-1])
c=d['configs']; print('$v', 'config5', c['config5']['value'], c['config5']['ms'], c['config5']['parity_vs_cpu'], 'call_gb', round(c['config5']['call_bytes']/1e9,2), 'config4', c['config4_rank0_of_8']['value'], c['config4_rank0_of_8']['ms'], c['config4_rank0_of_8']['parity_vs_cpu'])"
done
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_ld2.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; grep -E 'FAILED|Error|error' gpurun_out/$T/gpu_tests.log | head -20; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$T/gpu_tests.log
