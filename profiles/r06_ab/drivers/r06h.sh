# r06h: does the per-step RCCL collective of the N-GPU bench get CUs beside back-to-back renders?
# (a world of 1 over nccl on the one-GPU box; tools/gather_probe.py), NCCL stream at normal and high
# priority
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06h
mkdir -p gpurun_out/$T
timeout -k 10 300 python tools/gather_probe.py > gpurun_out/$T/probe.txt 2>&1 || { tail -20 gpurun_out/$T/probe.txt; exit 1; }
HIPRIO=1 MASTER_PORT=29532 timeout -k 10 300 python tools/gather_probe.py > gpurun_out/$T/probe_hiprio.txt 2>&1 || { tail -20 gpurun_out/$T/probe_hiprio.txt; exit 1; }
grep '^{' gpurun_out/$T/probe.txt gpurun_out/$T/probe_hiprio.txt
