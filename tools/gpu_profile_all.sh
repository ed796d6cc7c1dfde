# Full measurement of the current build on the GPU box (round-end evidence for profiles/):
#   PMC passes + summary (installed as profiles/pmc_summary.json first, so the bench line quotes
#   this build's counters), bench.py (default contract run), rocprofv3 kernel trace + stats.
# usage: bash tools/gpu_profile_all.sh <tag>      → gpurun_out/<tag>/
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
T=${1:-prof}
mkdir -p gpurun_out/$T
bash tools/pmc_profile.sh gpurun_out/$T/pmc || { echo PMC_FAILED; exit 3; }
# (pmc_profile.sh runs bench.py --steps 1 --warmup 1 per pass: two 1920x1080x512 calls)
python3 tools/pmc_summary.py gpurun_out/$T/pmc "yk_render_persistent<true, 0>" final42_1920x1080x512_d50_n1 gpurun_out/$T/pmc_summary.json 2123366400 > /dev/null || exit 4
python3 tools/pmc_summary.py gpurun_out/$T/pmc "yk_mt_warmup" final42_1920x1080x512_d50_n1 gpurun_out/$T/pmc_summary_warmup.json > /dev/null || exit 4
python3 tools/pmc_hbm.py gpurun_out/$T/pmc 1061683200 19 gpurun_out/$T/pmc_hbm.json > /dev/null || exit 4
cp gpurun_out/$T/pmc_summary.json profiles/pmc_summary.json
cp gpurun_out/$T/pmc_hbm.json profiles/pmc_hbm.json
timeout -k 10 400 python bench.py > gpurun_out/$T/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/$T/bench.log; exit 1; }
grep '^{' gpurun_out/$T/bench.log | tail -1 > gpurun_out/$T/bench.json
cat gpurun_out/$T/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/kt -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-modes --no-configs --no-tiles > gpurun_out/$T/kt.log 2>&1 || { echo KT_FAILED; tail -20 gpurun_out/$T/kt.log; exit 2; }
echo done
