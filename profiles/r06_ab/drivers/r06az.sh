# r06az: whole-image parity of the final build (packed candidate ids) of BASELINE config 3 (and config 4's rank-0 row tile) against the CPU
# oracle on every usable core (tools/full_parity.py)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r06az
timeout -k 10 1100 python -u tools/full_parity.py config3 config4 > gpurun_out/r06az/full_parity.log 2>&1 || { tail -20 gpurun_out/r06az/full_parity.log; exit 1; }
tail -3 gpurun_out/r06az/full_parity.log
