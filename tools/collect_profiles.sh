# Copy the judged evidence of one tools/gpu_round.sh / gpu_profile_all.sh run from gpurun_out/<tag>
# into profiles/ (tracked): bench line, rocprofv3 kernel stats + union of the render spans, PMC
# summary (also installed as profiles/pmc_summary.json, which bench.py reads), GPU test log tail.
set -e
T=$1
S=gpurun_out/$T
P=profiles
cp $S/bench.json $P/${T}_bench.json
cp $S/kt/run_kernel_stats.csv $P/${T}_kernel_stats.csv
# (the kt run of gpu_profile_all.sh: 2 warm-up + 6 timed steps of 512 spp, the first of each synced; the
# bench's in-flight launches are 64 spp, bench.py roofline.launch_ms)
python3 tools/kernel_union.py $S/kt/run_kernel_trace.csv "yk_render_persistent<true, 0>" $P/${T}_kernel_union.json ${KT_SPP:-4096} 64 8 > /dev/null
cp $S/pmc_summary.json $P/${T}_pmc_summary.json
cp $S/pmc_summary.json $P/pmc_summary.json
[ -f $S/pmc_summary_warmup.json ] && cp $S/pmc_summary_warmup.json $P/${T}_pmc_summary_warmup.json
[ -f $S/pmc_hbm.json ] && cp $S/pmc_hbm.json $P/${T}_pmc_hbm.json && cp $S/pmc_hbm.json $P/pmc_hbm.json
[ -f $S/gpu_tests.log ] && grep -E "PASSED|FAILED|SKIPPED|ERROR|passed|failed" $S/gpu_tests.log > $P/${T}_gpu_tests.txt || true
ls -la $P/${T}_*
