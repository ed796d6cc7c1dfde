# Parity of a variant (GPU parity/modes/group suites through YKGPU_LIB_OVERRIDE), the work counts
# of the variants (tools/quickbench.py through the same override), an A/B at one spp (FP64) and
# the same in the FP32 mode.
# usage: bash tools/gpu_h16.sh <tag> <variant-to-check> <spp> <variants...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; V=$2; SPP=$3; shift 3
mkdir -p gpurun_out/$T
L=$PWD/uecraytracing_amd/lib/abl
YKGPU_LIB_OVERRIDE=$L/libykgpu_$V.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modes.py tests/test_gpu_group.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/$T/parity_$V.log 2>&1 || { echo PARITY_FAILED; tail -30 gpurun_out/$T/parity_$V.log; exit 1; }
tail -1 gpurun_out/$T/parity_$V.log
for X in "$@"; do
  YKGPU_LIB_OVERRIDE=$L/libykgpu_$X.so timeout -k 10 120 python tools/quickbench.py final 1920x16 > gpurun_out/$T/qb_$X.txt 2>&1 || { echo QB_FAILED; tail -5 gpurun_out/$T/qb_$X.txt; exit 2; }
  echo "$X: $(tail -1 gpurun_out/$T/qb_$X.txt)"
done
timeout -k 10 900 python tools/abtime.py $SPP "$@" > gpurun_out/$T/ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab.txt; exit 3; }
cat gpurun_out/$T/ab.txt
AB_PREC=1 timeout -k 10 900 python tools/abtime.py $SPP "$@" > gpurun_out/$T/ab_f32.txt 2>&1 || { echo AB32_FAILED; tail -20 gpurun_out/$T/ab_f32.txt; exit 4; }
cat gpurun_out/$T/ab_f32.txt
