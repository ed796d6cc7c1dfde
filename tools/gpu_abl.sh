# Timing-only A/B of library variants (no parity: ablations are wrong by design).
# usage: bash tools/gpu_abl.sh <tag> <spp> <variants...>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=$1; SPP=$2; shift 2
mkdir -p gpurun_out/$T
timeout -k 10 900 python tools/abtime.py $SPP "$@" > gpurun_out/$T/ab.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab.txt; exit 2; }
cat gpurun_out/$T/ab.txt
