# r05aj: the render at the warm-up's issue priority (prio0: no s_setprio) against base (synced calls
# with image hashes, then bench steps, 3 rounds); then one PMC pass of LDS counters over a bench step of
# the production build (render kernel: bank-conflict cycles against LDS-array cycles, LDS issue stalls).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=r05aj
mkdir -p gpurun_out/$T
AB_REPS=2 timeout -k 10 300 python tools/abtime.py 512 base prio0 > gpurun_out/$T/ab512.txt 2>&1 || { echo AB_FAILED; tail -20 gpurun_out/$T/ab512.txt; exit 1; }
cat gpurun_out/$T/ab512.txt
for rnd in 0 1 2; do
  for v in base prio0; do
    if [ $v = base ]; then L=$PWD/uecraytracing_amd/lib/libykgpu.so; else L=$PWD/uecraytracing_amd/lib/abl/libykgpu_$v.so; fi
    YKGPU_LIB_OVERRIDE=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-modes --no-configs --no-tiles > gpurun_out/$T/bench_${v}_$rnd.log 2>&1 || { echo BENCH_FAILED $v; tail -5 gpurun_out/$T/bench_${v}_$rnd.log; exit 1; }
    python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/$T/bench_${v}_$rnd.log') if l.startswith('{')][-1])
print($rnd, '$v', d['value'], d['ms_per_step'])"
  done
done
PMC_GROUPS="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" timeout -k 10 400 bash tools/pmc_profile.sh gpurun_out/$T/pmc_lds || { echo PMC_FAILED; exit 1; }
python3 tools/pmc_summary.py gpurun_out/$T/pmc_lds "yk_render_persistent<true, 0>" final42_1920x1080x512_d50_n1 gpurun_out/$T/pmc_lds_render.json 2123366400 || exit 1
python3 tools/pmc_summary.py gpurun_out/$T/pmc_lds "yk_mt_warmup" final42_1920x1080x512_d50_n1 gpurun_out/$T/pmc_lds_warmup.json || exit 1
echo PMC_OK
