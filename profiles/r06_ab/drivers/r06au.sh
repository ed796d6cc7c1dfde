# r06au: the candidates' refined 1/a from the bounds' 1/a (YK_RA_FROM_IA, rafia: rcp_refined's first
# Newton step is rcp_bound's, bit for bit, so one step instead of rcp + two) against the product:
# parity, synced 512-spp A/B with image hashes, bench A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06au
mkdir -p gpurun_out/$T
YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_rafia.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/$T/parity_rafia.log 2>&1 || { echo PARITY_FAILED; grep -E "FAILED|Error" gpurun_out/$T/parity_rafia.log | head; tail -30 gpurun_out/$T/parity_rafia.log; exit 1; }
tail -1 gpurun_out/$T/parity_rafia.log
timeout -k 10 900 python tools/abtime.py 512 base rafia > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06au_bench base rafia || exit 3
