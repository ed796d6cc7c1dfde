# Phase split (stamp builds: -DYK_STAMPS=1, `make -C uecraytracing_amd/csrc stamps` → lib/abl/libykgpu_stamps.so) of lib/abl variants, on the GPU box.
# usage: bash tools/gpu_phases.sh <spp> <variant> ...
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
SPP=$1; shift
for v in "$@"; do
  echo "== $v"
  YKGPU_LIB_OVERRIDE=uecraytracing_amd/lib/abl/libykgpu_$v.so timeout -k 10 300 python -u tools/phases.py final $SPP || exit 1
done
