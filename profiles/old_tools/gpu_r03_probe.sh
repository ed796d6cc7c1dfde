# Round-3 first probe on the GPU box: VALU issue costs (tools/ubench.hip, the roofline peak's
# evidence) and configs 4/5 throughput of the current build.
# usage: bash tools/gpu_r03_probe.sh <tag>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-r03a}
mkdir -p gpurun_out/$T
timeout -k 10 180 tools/ubench gpurun_out/$T/ubench.jsonl > gpurun_out/$T/ubench.txt 2>&1 || { echo UBENCH_FAILED; tail -5 gpurun_out/$T/ubench.txt; exit 1; }
cat gpurun_out/$T/ubench.txt
timeout -k 10 300 python -u tools/configs45.py c4 c5 > gpurun_out/$T/configs45.txt 2>&1 || { echo C45_FAILED; tail -20 gpurun_out/$T/configs45.txt; exit 2; }
cat gpurun_out/$T/configs45.txt
