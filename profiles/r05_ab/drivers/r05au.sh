# r05au: the deferred unwind as the default (YK_UNWIND_DEFER=1): the GPU suite on the new build
# (base), then the full bench line (configs, modes) against head (the build before it), 2 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05au
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$T/gpu_tests.log
for rnd in 0 1; do
  for v in base head; do
    if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
    YKGPU_LIB_OVERRIDE=$L timeout -k 10 400 python bench.py --no-cpu-baseline --no-tiles > gpurun_out/$T/bench_${v}_$rnd.log 2>&1 || { echo BENCH_FAILED $v; tail -5 gpurun_out/$T/bench_${v}_$rnd.log; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/$T/bench_${v}_$rnd.log') if l.startswith('{')][-1])
print($rnd, '$v', d['value'], d['ms_per_step'], {k: (v['value'], v['parity_vs_cpu']['bytes_differing']) for k, v in d['configs'].items()}, {k: v['value'] for k, v in d['modes'].items()})"
  done
done
