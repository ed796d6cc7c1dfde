# r05ax: the unwind shared with the reduce only for launches of >= 16 spp (kUnwindMinKs; a whole
# config-4 frame's 8-spp launches keep the render's full unwind): the GPU suite on the new build
# (base), then a config-4 frame and config 3 synced against prev (before the shared unwind), and
# the full bench line (configs, modes), 2 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05ax
mkdir -p gpurun_out/$T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/$T/gpu_tests.log; exit 1; }
tail -2 gpurun_out/$T/gpu_tests.log
AB_W=3840 AB_REPS=2 timeout -k 10 500 python tools/abtime.py 1024 base prev > gpurun_out/$T/ab1024_w3840.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab1024_w3840.txt; exit 1; }
cat gpurun_out/$T/ab1024_w3840.txt
AB_REPS=2 timeout -k 10 300 python tools/abtime.py 512 base prev > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
for rnd in 0 1; do
  for v in base prev; do
    if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
    YKGPU_LIB_OVERRIDE=$L timeout -k 10 400 python bench.py --no-cpu-baseline --no-tiles > gpurun_out/$T/bench_${v}_$rnd.log 2>&1 || { echo BENCH_FAILED $v; tail -5 gpurun_out/$T/bench_${v}_$rnd.log; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/$T/bench_${v}_$rnd.log') if l.startswith('{')][-1])
print($rnd, '$v', d['value'], d['ms_per_step'], {k: (v['value'], v['parity_vs_cpu']['bytes_differing']) for k, v in d['configs'].items()}, {k: v['value'] for k, v in d['modes'].items()})"
  done
done
