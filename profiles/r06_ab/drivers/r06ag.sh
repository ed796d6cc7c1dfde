# r06ag: smoke of the r06ad tree; the FP64 visit's slab min / max two slots per asm block
# (YK_CULL_BLOCK, cullblk) and in-flight launches of 128 spp (YK_LAUNCH_SPP_OV=128, ov128; both:
# cullov) against the product: synced 512-spp A/B with image hashes, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06ag
mkdir -p gpurun_out/$T
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke: ok')" > gpurun_out/$T/smoke.txt 2>&1 || { tail -20 gpurun_out/$T/smoke.txt; exit 1; }
tail -1 gpurun_out/$T/smoke.txt
timeout -k 10 900 python tools/abtime.py 512 base cullblk > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06ag_bench base cullblk ov128 cullov || exit 3
