# r05az: the shared unwind compiled out (nou: -DYK_UNWIND_DEFER=0, same two-unit build) against base
# (shared for launches of >= 16 spp) and prev: a whole config-4 frame and config 3, synced, with image
# hashes; then bench lines with configs (3 rounds, base / nou).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05az
mkdir -p gpurun_out/$T
AB_W=3840 AB_REPS=2 timeout -k 10 500 python tools/abtime.py 1024 base nou prev > gpurun_out/$T/ab1024_w3840.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab1024_w3840.txt; exit 1; }
cat gpurun_out/$T/ab1024_w3840.txt
for rnd in 0 1 2; do
  for v in base nou; do
    if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
    YKGPU_LIB_OVERRIDE=$L timeout -k 10 400 python bench.py --no-cpu-baseline --no-tiles --no-modes > gpurun_out/$T/bench_${v}_$rnd.log 2>&1 || { echo BENCH_FAILED $v; tail -5 gpurun_out/$T/bench_${v}_$rnd.log; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/$T/bench_${v}_$rnd.log') if l.startswith('{')][-1])
print($rnd, '$v', d['value'], d['ms_per_step'], {k: (v['value'], v['parity_vs_cpu']['bytes_differing']) for k, v in d['configs'].items()})"
  done
done
