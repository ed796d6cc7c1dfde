set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/gpu_variant_ab.sh r03e split 512 base split || exit 1
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_split.so timeout -k 10 400 python bench.py --no-cpu-baseline --no-modes > gpurun_out/r03e/bench_split.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r03e/bench_split.log; exit 2; }
grep '^{' gpurun_out/r03e/bench_split.log | tail -1 | cut -c1-300
