# r06ar: the newest candidate's hb and disc kept from its leaf test (YK_CAND_HD: its exact root
# skips the second discriminant, 17 FP64 operations), at 112 VGPRs (hd, no spill) and 120 (hd120),
# against the product: parity of hd, synced 512-spp A/B with image hashes, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06ar
mkdir -p gpurun_out/$T
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_hd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/parity_hd.log 2>&1 || { echo PARITY_FAILED; grep -E "FAILED|Error" gpurun_out/$T/parity_hd.log | head; tail -30 gpurun_out/$T/parity_hd.log; exit 1; }
tail -1 gpurun_out/$T/parity_hd.log
timeout -k 10 900 python tools/abtime.py 512 base hd hd120 > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06ar_bench base hd hd120 || exit 3
