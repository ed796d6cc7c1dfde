# Builds lib/abl/libykgpu_<name>.so from a git revision's ykgpu_render.hip (same host objects and
# headers as the working tree): the A/B baseline of tools/abtime.py.
# usage: bash tools/build_head_variant.sh [rev] [name]
set -e
REV=${1:-HEAD}; NAME=${2:-head}
cd "$(dirname "$0")/../uecraytracing_amd/csrc"
mkdir -p ../lib/abl
git show "$REV":uecraytracing_amd/csrc/ykgpu_render.hip > _variant_render.hip
/opt/rocm/bin/hipcc -std=c++17 -O3 -ffp-contract=off -fno-fast-math -fPIC --offload-arch=gfx950 -c -o ../lib/abl/r_$NAME.o _variant_render.hip
rm -f _variant_render.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/abl/libykgpu_$NAME.so ../lib/abl/r_$NAME.o ../lib/yk_host.o ../lib/yk_bvh.o
