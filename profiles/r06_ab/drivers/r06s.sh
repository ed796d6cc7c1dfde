# r06s: the FP64 unwind without spill checks when no ending lane of the wave spilled (two ids per
# round: YK_UNWIND_FAST) vs the product (branch-free visit); parity suite, synced A/B at 512 spp,
# bench A/B; then the product's LDS counters (one PMC pass over a 1-step bench)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r06s
mkdir -p gpurun_out/$T
for V in unwf; do
  YKGPU_LIB_OVERRIDE=$PWD/uecraytracing_amd/lib/abl/libykgpu_$V.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_modes.py -m gpu -x -v --timeout 100 --timeout-method thread > gpurun_out/$T/parity_$V.log 2>&1 || { echo PARITY_FAILED $V; tail -30 gpurun_out/$T/parity_$V.log; exit 1; }
  echo $V; tail -1 gpurun_out/$T/parity_$V.log
done
timeout -k 10 900 python tools/abtime.py 512 base unwf base unwf > gpurun_out/$T/ab512.txt 2>&1 || { tail -20 gpurun_out/$T/ab512.txt; exit 2; }
cat gpurun_out/$T/ab512.txt
bash tools/gpu_bench_ab.sh r06s_bench base unwf || exit 3
PMC_GROUPS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" bash tools/pmc_profile.sh gpurun_out/$T/pmc_lds || { echo PMC_FAILED; exit 4; }
python3 tools/pmc_summary.py gpurun_out/$T/pmc_lds "yk_render_persistent<true, 0>" final42_1920x1080x512_d50_n1 gpurun_out/$T/pmc_lds_summary.json > /dev/null && cat gpurun_out/$T/pmc_lds_summary.json
