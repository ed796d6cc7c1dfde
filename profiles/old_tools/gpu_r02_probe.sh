# Round-2 probe on the GPU box: host CPU share, counter list, FP64/FP32 flop-counter calibration
# (tools/flopcal), and the render kernel's FP64 instruction mix under the same counters.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r02_probe
mkdir -p $O
{ nproc; python3 -c 'import os; print("cpu_count", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)))'
  cat /sys/fs/cgroup/cpu.max 2>/dev/null; cat /sys/fs/cgroup/pids.max 2>/dev/null; lscpu | head -20; } > $O/host.txt 2>&1
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || echo "list rc $?"
grep -o "SQ_[A-Z0-9_]*F64[A-Z0-9_]*\|SQ_INSTS_VALU_FLOPS[A-Z0-9_]*\|SQ_[A-Z_]*TRANS[A-Z0-9_]*" $O/counters.txt | sort -u > $O/f64_counters.txt || true
cat $O/f64_counters.txt
timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU --output-format csv -d $O/cal1 -o run -- tools/flopcal > $O/cal1.log 2>&1 || { echo CAL1_FAILED; exit 1; }
# the per-op F64 counters, when the list has them (at most 8 SQ counters in one pass)
C2=""
for c in SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32; do
  grep -qx "$c" $O/f64_counters.txt && C2="$C2 $c"
  grep -qw "$c" $O/counters.txt && ! echo "$C2" | grep -qw "$c" && C2="$C2 $c"
done
echo "pass2: $C2"
if [ -n "$C2" ]; then
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $C2 --output-format csv -d $O/cal2 -o run -- tools/flopcal > $O/cal2.log 2>&1 || { echo CAL2_FAILED; exit 1; }
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C2 --output-format csv -d $O/render2 -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-modes > $O/render2.log 2>&1 || { echo RENDER2_FAILED; exit 1; }
fi
echo PROBE_OK
