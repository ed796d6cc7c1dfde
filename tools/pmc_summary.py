"""Summarise tools/pmc_profile.sh output: per-kernel counters averaged per dispatch."""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
kern = sys.argv[2] if len(sys.argv) > 2 else "yk_render_persistent"
agg = collections.defaultdict(float)
disp = collections.defaultdict(set)
dur = []
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
for f in sorted(glob.glob(os.path.join(d, "p*", "run_kernel_trace.csv"))):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            dur.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
per = {k: v / len(disp[k]) for k, v in agg.items()}
out = {"kernel": kern, "dispatches_profiled": len(dur), "mean_ms": sum(dur) / max(1, len(dur)), "counters_per_dispatch": per}
if "SQ_THREAD_CYCLES_VALU" in per and "SQ_ACTIVE_INST_VALU" in per:
    out["valu_lane_utilization"] = per["SQ_THREAD_CYCLES_VALU"] / (per["SQ_ACTIVE_INST_VALU"] * 64)
if "SQ_WAVE_CYCLES" in per:
    wc = per["SQ_WAVE_CYCLES"]
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in per:
            out[k + "_frac"] = per[k] / wc
if "FETCH_SIZE" in per:
    out["hbm_bytes_fetch_corrected"] = per["FETCH_SIZE"] * 1024 * 2  # gfx950: FETCH_SIZE reads 1/2 (MICROARCH §HBM)
if "WRITE_SIZE" in per:
    out["hbm_bytes_write"] = per["WRITE_SIZE"] * 1024
print(json.dumps(out, indent=1))
