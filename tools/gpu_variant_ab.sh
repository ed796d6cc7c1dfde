# Parity of a library variant (the GPU parity suite through YKGPU_LIB_OVERRIDE), then an A/B of
# variants at one spp (tools/abtime.py), then optional extra commands.
# usage: bash tools/gpu_variant_ab.sh <tag> <variant-to-check> <spp> <variants...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; V=$2; SPP=$3; shift 3
mkdir -p gpurun_out/$T
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_$V.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modes.py tests/test_gpu_group.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$T/parity_$V.log 2>&1 || { echo PARITY_FAILED; tail -30 gpurun_out/$T/parity_$V.log; exit 1; }
tail -1 gpurun_out/$T/parity_$V.log
timeout -k 10 900 python tools/abtime.py $SPP "$@" > gpurun_out/$T/ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab.txt; exit 2; }
cat gpurun_out/$T/ab.txt
