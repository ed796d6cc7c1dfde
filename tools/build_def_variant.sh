# Builds lib/abl/libykgpu_<name>.so from the working tree's ykgpu_render.hip with extra -D flags
# (same host objects as lib/): an A/B variant of tools/abtime.py.  Like lib/libykgpu.so, two units:
# everything but the FP32 render kernel, and the FP32 render kernel under max-ilp (YK_SPLIT);
# SPLIT=0 builds one unit (every kernel under the default scheduler).
# usage: [SPLIT=0] bash tools/build_def_variant.sh <name> -DNAME=VALUE [...]
set -e
NAME=$1; shift
cd "$(dirname "$0")/../uecraytracing_amd/csrc"
mkdir -p ../lib/abl
F="-std=c++17 -O3 -ffp-contract=off -fno-fast-math -fPIC --offload-arch=gfx950"
if [ "${SPLIT:-1}" = 0 ]; then
  /opt/rocm/bin/hipcc $F "$@" -c -o ../lib/abl/r_$NAME.o ykgpu_render.hip
  OBJS=../lib/abl/r_$NAME.o
else
  /opt/rocm/bin/hipcc $F -DYK_SPLIT=1 "$@" -c -o ../lib/abl/r_$NAME.o ykgpu_render.hip &
  /opt/rocm/bin/hipcc $F -DYK_SPLIT=2 -mllvm --amdgpu-sched-strategy=max-ilp -Wno-unused-function \
    -Wno-unused-const-variable "$@" -c -o ../lib/abl/r32_$NAME.o ykgpu_render.hip &
  wait
  OBJS="../lib/abl/r_$NAME.o ../lib/abl/r32_$NAME.o"
fi
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../lib/abl/libykgpu_$NAME.so $OBJS ../lib/yk_host.o ../lib/yk_bvh.o
rm -f $OBJS
echo "built lib/abl/libykgpu_$NAME.so ($*)"
