# bench.py (no CPU baseline, no modes) once per variant, interleaved twice; a variant is a library
# (base = lib/libykgpu.so, else lib/abl/libykgpu_<name>.so) with optional "@VAR=value" settings.
# usage: bash tools/gpu_bench_ab.sh <tag> <variant> ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; shift
mkdir -p gpurun_out/$T
for rnd in 0 1; do
  i=0
  for spec in "$@"; do
    i=$((i+1))
    IFS='@' read -r -a parts <<< "$spec"
    v=${parts[0]}
    if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
    envs=("YKGPU_LIB_OVERRIDE=$L")
    for e in "${parts[@]:1}"; do envs+=("$e"); done
    env "${envs[@]}" timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes --no-configs --no-tiles > gpurun_out/$T/bench_${i}_$rnd.log 2>&1 || { echo BENCH_FAILED $spec; tail -5 gpurun_out/$T/bench_${i}_$rnd.log; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/$T/bench_${i}_$rnd.log') if l.startswith('{')][-1])
b=d['roofline']['step_breakdown_ms']
print($rnd, '$spec', d['value'], d['ms_per_step'], 'busy', b['render_busy'], 'reduce', b['reduce'], 'warm', b['mt_warmup'])"
  done
done
