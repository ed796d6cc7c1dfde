# r06al: an in-flight call of one launch keeps the rings' full depth (YK_INFLIGHT_DEEP, deep): the
# 8-way tile of config 3 (132.7M slots) then runs ONE 512-spp launch per in-flight call, overlapping
# the calls around it like the frame's launches, instead of two of 256 — the robustness suite on the
# variant library, tile A/Bs (20 back-to-back calls), bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06al
mkdir -p gpurun_out/$T
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_deep.so timeout -k 10 600 python -u -m pytest tests/test_gpu_robust.py tests/test_gpu_group.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/robust_deep.log 2>&1 || { echo ROBUST_FAILED; grep -E "FAILED|Error" gpurun_out/$T/robust_deep.log | head; tail -30 gpurun_out/$T/robust_deep.log; exit 1; }
tail -1 gpurun_out/$T/robust_deep.log
for TL in 1920:512:8:0:rows 1920:512:8:7:rows 1920:512:4:0:rows; do
  TILE=$TL CALLS=20 timeout -k 10 600 python tools/tile_ab.py base deep > gpurun_out/$T/tile_${TL//:/_}.txt 2>&1 || { tail -20 gpurun_out/$T/tile_${TL//:/_}.txt; exit 2; }
  echo "== $TL"; cat gpurun_out/$T/tile_${TL//:/_}.txt
done
bash tools/gpu_bench_ab.sh r06al_bench base deep || exit 3
