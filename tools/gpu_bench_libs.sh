# The contract bench (FP64 headline only: no CPU baseline, modes or configs) run with several
# library variants in turn, twice, on one box: a same-box comparison of the bench line itself.
# usage: bash tools/gpu_bench_libs.sh <tag> <variant> ...   (lib/abl/libykgpu_<variant>.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; shift
mkdir -p gpurun_out/$T
for r in 1 2; do
  for v in "$@"; do
    YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-modes --no-configs --steps 5 > gpurun_out/$T/b_${v}_$r.log 2>&1 || { echo BENCH_FAILED $v; tail -5 gpurun_out/$T/b_${v}_$r.log; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('gpurun_out/$T/b_${v}_$r.log') if l.startswith('{')][-1]);b=d['roofline']['step_breakdown_ms'];print('$r $v', d['value'], d['ms_per_step'], b['render_busy'], b['reduce'])"
  done
done
