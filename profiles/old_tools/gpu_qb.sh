# quickbench (work counters) of the current library and of lib/abl variants, on the GPU box.
# usage: bash tools/gpu_qb.sh "<sizes>" <variant> ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
SIZES=$1; shift
for v in base "$@"; do
  if [ $v = base ]; then L=uecraytracing_amd/lib/libykgpu.so; else L=uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
  echo "== $v"
  YKGPU_LIB_OVERRIDE=$L timeout -k 10 300 python -u tools/quickbench.py final $SIZES || exit 1
done
