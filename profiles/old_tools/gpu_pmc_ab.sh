# One rocprofv3 PMC pass over quickbench (1920x32, final scene) per library variant.
# usage: bash tools/gpu_pmc_ab.sh "<counters>" <variant> ...   (variant base = lib/libykgpu.so)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcab
CTR=$1; shift
for v in "$@"; do
  if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
  YKGPU_LIB_OVERRIDE=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CTR --output-format csv -d gpurun_out/pmcab/$v -o run -- python3 tools/quickbench.py final 1920x32 > gpurun_out/pmcab/$v.log 2>&1 || { echo FAIL $v; tail -20 gpurun_out/pmcab/$v.log; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/pmcab/$v yk_render_persistent > gpurun_out/pmcab/$v.json || exit 2
  echo "== $v"; python3 -c "
import json; d=json.load(open('gpurun_out/pmcab/$v.json')); c=d['counters_per_dispatch']; print('mean_ms', round(d['mean_ms'],2)); [print(k, '%.4g'%v) for k,v in sorted(c.items())]"
done
