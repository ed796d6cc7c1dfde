# r05ae: the adopted candidate (ilp4: the deferred warm-up walking four slots per lane at 48 VGPRs,
# the grid trimmed to a multiple of four) and inl4 (the same, plus four walks per lane in the
# in-line warm-ups: config 5's, FP32's, lens-free scenes') against base: synced calls with image
# hashes, then the full bench line (configs and modes) per variant, 2 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05ae
mkdir -p gpurun_out/$T
AB_REPS=2 timeout -k 10 400 python tools/abtime.py 512 base ilp4 inl4 > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
for rnd in 0 1; do
  for v in base ilp4 inl4; do
    if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
    YKGPU_LIB_OVERRIDE=$L timeout -k 10 400 python bench.py --no-cpu-baseline --no-tiles > gpurun_out/$T/bench_${v}_$rnd.log 2>&1 || { echo BENCH_FAILED $v; tail -5 gpurun_out/$T/bench_${v}_$rnd.log; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/$T/bench_${v}_$rnd.log') if l.startswith('{')][-1])
c=d.get('configs',{}); m=d.get('modes',{})
print($rnd, '$v', d['value'], d['ms_per_step'], {k: (v['value'], v['parity_vs_cpu']['bytes_differing']) for k, v in c.items()}, {k: v['value'] for k, v in m.items()})"
  done
done
