# r05as: the deferred warm-up's grid with four walks per lane (YKGPU_WARM_PER_CU on the -DYK_AB_KNOBS build):
# 8 / 16 / 64 blocks per CU against the default 32 (knobs with no variable, and base; at 8 the waves hold
# > 4096 slots and the in-line warm-up runs): synced calls with image hashes, then
# bench steps (2 rounds).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05as
mkdir -p gpurun_out/$T
AB_REPS=2 timeout -k 10 400 python tools/abtime.py 512 base knobs knobs@YKGPU_WARM_PER_CU=8 knobs@YKGPU_WARM_PER_CU=16 knobs@YKGPU_WARM_PER_CU=64 > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
K=$PWD/uecraytracing_amd/lib/abl/libykgpu_knobs.so
for rnd in 0 1; do
  for v in base k0 k8 k16 k64; do
    case $v in base) L=$PWD/uecraytracing_amd/lib/libykgpu.so; E="";; k0) L=$K; E="";; *) L=$K; E="YKGPU_WARM_PER_CU=${v#k}";; esac
    env $E YKGPU_LIB_OVERRIDE=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes --no-configs --no-tiles > gpurun_out/$T/bench_${v}_$rnd.log 2>&1 || { echo BENCH_FAILED $v; tail -5 gpurun_out/$T/bench_${v}_$rnd.log; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/$T/bench_${v}_$rnd.log') if l.startswith('{')][-1])
print($rnd, '$v', d['value'], d['ms_per_step'])"
  done
done
