# r05aw: a whole config-4 frame (3840x2160x1024, 128 launches of 8 spp) with the unwind shared with
# the reduce (base) against the build before it (prev): the bench's tiles line put the frame at
# 1459.8 ms against 1350.9 in r05ao, while the tiles got faster. Synced calls with image hashes,
# then the same for config 3 at 1920 (control).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05aw
mkdir -p gpurun_out/$T
AB_W=3840 AB_REPS=2 timeout -k 10 500 python tools/abtime.py 1024 base prev > gpurun_out/$T/ab1024_w3840.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab1024_w3840.txt; exit 1; }
cat gpurun_out/$T/ab1024_w3840.txt
AB_REPS=2 timeout -k 10 300 python tools/abtime.py 512 base prev > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
