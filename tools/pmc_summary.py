"""Summarise tools/pmc_profile.sh output for one kernel: counters per dispatch and derived
metrics (gfx950 corrections per MI355X_MICROARCH.md §HBM: FETCH_SIZE reads half of a wide
stream; GRBM_GUI_ACTIVE sums the 8 XCDs; SQ_* cycle counters are quad-cycles).
usage: python tools/pmc_summary.py <pmc dir> [kernel-substring[|substring...]] [workload-tag] [out.json]
                                  [samples rendered by the profiled dispatches]
Several '|'-separated substrings (kernels that share a launch) sum their counters; "per dispatch"
then means per dispatch of the LAST one (one per launch).
VALU busy / lane utilisation / the wait fractions come from the summed counters too."""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "yk_render_persistent"
workload = sys.argv[3] if len(sys.argv) > 3 else None
names = kern.split("|")
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
dur = []
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if any(k in r["Kernel_Name"] for k in names):
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            if names[-1] in r["Kernel_Name"]:
                disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
for f in sorted(glob.glob(os.path.join(d, "p*", "run_kernel_trace.csv"))):
    for r in csv.DictReader(open(f)):
        if names[-1] in r["Kernel_Name"]:
            dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
per = {k: v / max(1, len(disp[k])) for k, v in agg.items()}
out = {"source": f"rocprofv3 --kernel-trace --pmc (4 passes), {d}", "kernel": kern,
       "workload": workload, "dispatches_profiled": len(dur),
       "mean_ms": sum(dur) / max(1, len(dur)), "counters_per_dispatch": per}
if "SQ_THREAD_CYCLES_VALU" in per and "SQ_ACTIVE_INST_VALU" in per:
    out["valu_lane_utilization"] = per["SQ_THREAD_CYCLES_VALU"] / (per["SQ_ACTIVE_INST_VALU"] * 64)
if "SQ_ACTIVE_INST_VALU" in per and "GRBM_GUI_ACTIVE" in per:
    cycles = per["GRBM_GUI_ACTIVE"] / 8  # per XCD
    out["valu_busy"] = per["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * cycles)
if "SQ_WAVE_CYCLES" in per:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in per:
            out[k + "_frac"] = per[k] / per["SQ_WAVE_CYCLES"]
if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
    out["hbm_bytes_per_launch"] = per["FETCH_SIZE"] * 1024 * 2 + per["WRITE_SIZE"] * 1024
    if len(sys.argv) > 5:
        # per sample: the FETCH_SIZE pass's and the WRITE_SIZE pass's dispatches each render the
        # given samples (one bench run per pass)
        tot = (agg["FETCH_SIZE"] * 1024 * 2 + agg["WRITE_SIZE"] * 1024)
        out["samples_per_pass"] = int(float(sys.argv[5]))
        out["hbm_bytes_per_sample"] = tot / out["samples_per_pass"]
if "SQ_INSTS_VALU" in per and "GRBM_GUI_ACTIVE" in per:
    # SIMD-32: a wave64 VALU instruction holds its SIMD 2 cycles (MI355X_MICROARCH.md)
    out["valu_pipe_util"] = per["SQ_INSTS_VALU"] * 2 / (1024 * per["GRBM_GUI_ACTIVE"] / 8)
if "SQ_LDS_BANK_CONFLICT" in per and "SQ_LDS_IDX_ACTIVE" in per:
    out["lds_bank_conflict_frac"] = per["SQ_LDS_BANK_CONFLICT"] / max(1.0, per["SQ_LDS_IDX_ACTIVE"])
if "SQ_LDS_IDX_ACTIVE" in per and "GRBM_GUI_ACTIVE" in per:
    out["lds_array_busy"] = per["SQ_LDS_IDX_ACTIVE"] / (256 * per["GRBM_GUI_ACTIVE"] / 8)
if "SQ_INSTS_VALU_FLOPS_FP64" in per:
    out["fp64_flops_hw_per_launch"] = per["SQ_INSTS_VALU_FLOPS_FP64"]
js = json.dumps(out, indent=1)
if len(sys.argv) > 4:
    open(sys.argv[4], "w").write(js + "\n")
print(js)
