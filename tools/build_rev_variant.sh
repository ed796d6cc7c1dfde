# Builds lib/abl/libykgpu_<name>.so entirely from a git revision (kernel, host objects and
# headers of that revision): the A/B baseline when the change touches host code or shared layouts.
# usage: bash tools/build_rev_variant.sh [rev] [name]
set -e
REV=${1:-HEAD}; NAME=${2:-rev}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
TMP=$(mktemp -d)
git -C "$ROOT" archive "$REV" uecraytracing_amd/csrc include | tar -x -C "$TMP"
cd "$TMP/uecraytracing_amd/csrc"
F="-std=c++17 -O3 -ffp-contract=off -fno-fast-math -fPIC"
/opt/rocm/bin/hipcc $F --offload-arch=gfx950 -c -o r.o ykgpu_render.hip
g++ $F -c -o h.o yk_host.cpp
g++ $F -c -o b.o yk_bvh.cpp
mkdir -p "$ROOT/uecraytracing_amd/lib/abl"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/uecraytracing_amd/lib/abl/libykgpu_$NAME.so" r.o h.o b.o
rm -rf "$TMP"
echo "built lib/abl/libykgpu_$NAME.so from $REV"
