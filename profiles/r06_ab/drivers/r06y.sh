# r06y: launch sizes on the current build (r06v + dielectric precompute): frame launches of 64 spp
# (l64: 8 per frame), 64 with a first synced launch of 8 (l64f8), 48 (l48), and 64 with tile
# launches of 2^27 slots (l64s27); synced A/B at 512 spp, bench A/B (launch sizes change no
# arithmetic: the images' hashes are compared)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06y
mkdir -p gpurun_out/$T
timeout -k 10 900 python tools/abtime.py 512 base l64 l64f8 l48 l64s27 > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06y_bench base l64 l64f8 l48 l64s27 || exit 3
