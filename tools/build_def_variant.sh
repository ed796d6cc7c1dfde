# Builds lib/abl/libykgpu_<name>.so from the working tree's ykgpu_render.hip with extra -D flags
# (same host objects as lib/): an A/B variant of tools/abtime.py.
# usage: bash tools/build_def_variant.sh <name> -DNAME=VALUE [...]
set -e
NAME=$1; shift
cd "$(dirname "$0")/../uecraytracing_amd/csrc"
mkdir -p ../lib/abl
/opt/rocm/bin/hipcc -std=c++17 -O3 -ffp-contract=off -fno-fast-math -fPIC --offload-arch=gfx950 "$@" -c -o ../lib/abl/r_$NAME.o ykgpu_render.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/abl/libykgpu_$NAME.so ../lib/abl/r_$NAME.o ../lib/yk_host.o ../lib/yk_bvh.o
rm -f ../lib/abl/r_$NAME.o
echo "built lib/abl/libykgpu_$NAME.so ($*)"
