"""Summarise tools/gpu_fp64_reconcile.sh output into one JSON.

usage: python tools/fp64_reconcile_summary.py <dir> [out.json]
  <dir>/cal  : rocprofv3 --pmc over tools/flopcal (known instruction counts)
  <dir>/rec  : rocprofv3 --pmc over tools/fp64_reconcile.py (all lanes, then one lane per wave)
  <dir>/rec_counts.json : the two calls' work counters
"""
import collections
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from uecraytracing_amd import flops  # noqa: E402


def per_dispatch(path):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    name = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        agg[d][r["Counter_Name"]] += float(r["Counter_Value"])
        name[d] = r["Kernel_Name"]
    return [(name[d], dict(agg[d])) for d in sorted(agg)]


def main():
    d = sys.argv[1]
    cal_cases = [ln.split() for ln in open(os.path.join(d, "cal.log")) if ln.startswith("case ")]
    cal = []
    disp = [x for x in per_dispatch(os.path.join(d, "cal", "run_counter_collection.csv")) if "cal<" in x[0]]
    for case, (kname, c) in zip(cal_cases, disp):
        wave_instr = float(case[5])
        cal.append({"op": case[1], "active_lanes": int(case[3]),
                    "flops_fp64_per_wave_instr": round(c["SQ_INSTS_VALU_FLOPS_FP64"] / wave_instr, 3),
                    "lane_util": round(c["SQ_THREAD_CYCLES_VALU"] / (64 * c["SQ_ACTIVE_INST_VALU"]), 3)})
    rc = json.load(open(os.path.join(d, "rec_counts.json")))
    ren = [c for n, c in per_dispatch(os.path.join(d, "rec", "run_counter_collection.csv"))
           if "yk_render_persistent" in n or "yk_render_counting" in n]
    assert len(ren) == 2, "expected two render dispatches (all lanes, one lane)"
    st = rc["calls"][0]
    assert all(rc["calls"][1][k] == st[k] for k in st if k != "flags"), "calls did different work"
    full, one = ren
    issued = full["SQ_INSTS_VALU_FLOPS_FP64"] * 64       # lane-slots of the FP64 instructions issued
    executed = one["SQ_INSTS_VALU_FLOPS_FP64"]           # one lane per wave: executed operations
    alg = flops.algorithmic(st)
    impl = flops.implementation(st)
    out = {
        "workload": rc["workload"],
        "calibration": {
            "finding": "SQ_INSTS_VALU_FLOPS_FP64 counts once per wave-instruction whatever the exec "
                       "mask (FMA and div_fmas 2, add/mul/rcp 1; cmp/max/cvt/ldexp/div_scale/"
                       "div_fixup 0): lane flops = counter x active lanes, not the counter",
            "cases": cal},
        "work": st,
        "samples": st["samples"],
        "issued_lane_slots_fp64": issued,
        "executed_fp64_one_lane_counter": executed,
        "model_implementation": impl,
        "model_algorithmic": alg,
        "implementation_model_vs_counter": round(impl / executed, 4),
        "algorithmic_share_of_executed": round(alg / executed, 4),
        "fp64_lane_utilization": round(executed / issued, 4),
        "kernel_lane_utilization_all_valu": round(full["SQ_THREAD_CYCLES_VALU"] / (64 * full["SQ_ACTIVE_INST_VALU"]), 4),
        "per_sample": {"algorithmic": round(alg / st["samples"], 1), "implementation_model": round(impl / st["samples"], 1),
                       "executed_counter": round(executed / st["samples"], 1),
                       "issued_lane_slots": round(issued / st["samples"], 1)},
        "images_equal": rc["images_equal"],
    }
    js = json.dumps(out, indent=1)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
