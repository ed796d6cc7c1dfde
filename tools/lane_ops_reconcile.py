"""Reconciles the VALU lane-op models with the PMC counters.

usage: python tools/lane_ops_reconcile.py <probe pmc dir> <probe.json> <out.json>

<probe pmc dir> holds rocprofv3 --pmc passes (p*/run_counter_collection.csv) over
tools/lane_ops_probe.py: calls A (production), B (counting), C (counting, one lane per wave) of
the same samples.  Per kernel:

* PMC-derived executed lane-ops = SQ_INSTS_VALU x 64 x lane utilisation, with the utilisation
  SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU) (the SQ counters count wave-instructions
  whatever the exec mask: tools/flopcal.hip, profiles/r02_fp64_reconcile.json).
* yk_render_persistent — the model is the one-lane count: in call C every wave runs one lane, so
  SQ_INSTS_VALU is exactly the instructions the lanes executed for these samples.  It must agree
  with call B's PMC-derived lane-ops (the same binary and samples, all lanes) within 10%.  The
  production instance (call A) is another binary: no counters, and held at 128 VGPRs where the
  counting instance is not, so it issues fewer instructions for the same samples — the ratio of
  the two calls' wave-instruction counts (SQ_INSTS_VALU, same samples and lane masks) carries the
  one-lane count over to it, and call A's PMC figure checks that within 10%.  (The counters' own
  adds, one per counted event, are only part of the difference: counting_increments_per_sample.)
* the warm-up — the model is the kernel's instruction count per sample read off its ISA
  (hipcc --cuda-device-only -S, VALU per basic block), times the lanes that run each block:
  - yk_mt_warmup<true, false> (the rejection loop in line, WARM_*): the index math and seed (31
    VALU), the walk loop (12 VALU per 4 steps, 99 trips), the rest of the start's draws and the
    camera ray (146), and 108 per thin-lens rejection iteration (4 words each: the iterations are
    (start words - 4) / 4 per sample, from the work counters);
  - yk_mt_warmup_defer (the retries drawn after the walks, DEFER["k1"]; round 5's production warm-up
    for launches of <= 4096 slots per wave): per sample the loop body through the first
    candidate (1424: index math, seed, walk, the start's draws, the candidate, the latch), then
    the camera ray and StartRec (48) for a sample accepted there or the ring store (10) for one
    rejected; per retry the ring read and the candidate (7 + 9 + 106), then the ring store (9) or
    the camera ray (71).  Rejections at the first candidate are taken at their expectation
    (1 - pi/4 per sample); every retry ends a rejection, so retries = candidates - samples.
    Since r05af the kernel walks four slots per lane (DEFER["k4"], the default; YK_DEFER_MODEL=k1
    re-reads the r05v passes with the one-walk build's counts).
* The algorithmic lane-ops (uecraytracing_amd/flops.py lane_ops) over the executed ones: how much
  of what the VALU executes is the reference's own arithmetic.
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from uecraytracing_amd import flops  # noqa: E402

# yk_mt_warmup<true, false> VALU instructions (ISA block counts, see the docstring)
WARM_FIXED = 26 + 5 + 31 + 115
WARM_WALK_LOOP = 12 * 99
WARM_LENS_ITER = 108

# yk_mt_warmup_defer (VALU per basic block, see the docstring), per build:
#  "k1" (r05v: one walk per lane):
#  "k4" (since r05af: four walks per lane): per 4-slot trip the four slots' index math and seed
#       (117), the walks' first step (14) and loop (48 per 4 steps, 99 trips), the first slot's
#       start through its candidate (203), for each of the other three its index math and seed
#       again (26) and its start (206), the latch (4); per sample accepted at once the camera ray
#       and StartRec (52 + 2), per rejection the ring store (10 + 1); the drain as k1 but the
#       camera ray (74)
DEFER = {
    "k1": dict(main=23 + 3 + 5 + 12 * 99 + 200 + 3 + 2, finish_main=48, put_main=10, retry=7 + 9 + 106,
               put_retry=9, finish_retry=71),
    "k4": dict(main=(117 + 14 + 48 * 99 + 203 + 3 * (26 + 206) + 4) / 4.0, finish_main=54, put_main=11,
               retry=122, put_retry=9, finish_retry=74),
}
DEFER_BUILD = os.environ.get("YK_DEFER_MODEL", "k4")
P_REJECT = 1.0 - 3.141592653589793 / 4.0

RENDER = "yk_render_persistent<true, "
COUNTING = "yk_render_counting<true, "  # the counting instances (round 6: a kernel name of their own)
WARM = "yk_mt_warmup"  # yk_mt_warmup<true, false> or yk_mt_warmup_defer


def dispatches(pmc_dir):
    """{(pass, dispatch id): {'kernel': name, counter: value}} in dispatch order per pass."""
    out = collections.OrderedDict()
    for f in sorted(glob.glob(os.path.join(pmc_dir, "p*", "run_counter_collection.csv"))):
        p = os.path.basename(os.path.dirname(f))
        for r in csv.DictReader(open(f)):
            key = (p, int(r["Dispatch_Id"]))
            d = out.setdefault(key, {"kernel": r["Kernel_Name"]})
            d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return out


def per_call(disp, kernel, ncalls):
    """Sums the counters of `kernel`'s dispatches, split into `ncalls` equal consecutive groups per
    pass (the probe's calls, in order), merged over the passes."""
    calls = [collections.defaultdict(float) for _ in range(ncalls)]
    by_pass = collections.defaultdict(list)
    for (p, _), d in disp.items():
        if kernel in d["kernel"]:
            by_pass[p].append(d)
    for p, ds in by_pass.items():
        if len(ds) % ncalls:
            raise SystemExit(f"{p}: {len(ds)} dispatches of {kernel} do not split into {ncalls} calls")
        n = len(ds) // ncalls
        for c in range(ncalls):
            for d in ds[c * n:(c + 1) * n]:
                for k, v in d.items():
                    if k != "kernel":
                        calls[c][k] += v
    return calls


def executed(c):
    lu = c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"])
    return c["SQ_INSTS_VALU"] * 64.0 * lu, lu


def count_increments(st):
    """VALU adds the counting instance spends on its counters for this work (one per event)."""
    w = st["work"]
    return (st["segments"] + st["sphere_tests"] + st["node_visits"] + st["sqrt_calls"] + st["newton_calls"]
            + st["newton_iters"] + w[0] + w[1] + w[2] + w[3] + w[4] + st["linear_scans"] + 3 * st["samples"])


def main():
    pmc_dir, probe, out = sys.argv[1:4]
    pr = json.load(open(probe))
    st = next(c for c in pr["calls"] if c["call"] == "B")
    n = st["samples"]
    disp = dispatches(pmc_dir)
    # render: production (A) is yk_render_persistent<true, 0>; B and C are both yk_render_counting<true, 1>
    ra = per_call(disp, RENDER + "0>", 1)[0]
    rb, rc = per_call(disp, COUNTING + "1>", 2)
    wa, wb, wc = per_call(disp, WARM, 3)
    e_a, lu_a = executed(ra)
    e_b, lu_b = executed(rb)
    one = rc["SQ_INSTS_VALU"]  # call C: one lane per wave, so wave-instructions = lane-instructions
    inc = count_increments(st)
    lo = flops.lane_ops(st)
    alg_r = sum(lo["render"].values())
    alg_w = sum(lo["warmup"].values())
    swords = st["work"][6]
    lens_iters = max(0.0, (swords - 4.0 * n) / 4.0)  # thin-lens candidates per sample x samples
    defer = any("yk_mt_warmup_defer" in d["kernel"] for d in disp.values())
    if defer:
        rej1 = P_REJECT * n
        retries = max(0.0, lens_iters - n)
        m = DEFER[DEFER_BUILD]
        warm_model = (n * m["main"] + (n - rej1) * m["finish_main"] + rej1 * m["put_main"]
                      + retries * m["retry"] + (retries - rej1) * m["put_retry"] + rej1 * m["finish_retry"])
    else:
        warm_model = n * (WARM_FIXED + WARM_WALK_LOOP) + lens_iters * WARM_LENS_ITER
    e_w, lu_w = executed(wa)
    res = {
        "workload": pr["workload"], "samples": n, "images_equal": pr["images_equal"],
        "source": f"rocprofv3 --pmc over tools/lane_ops_probe.py ({os.path.relpath(pmc_dir, ROOT)})",
        "render": {
            "pmc_executed_lane_ops_per_sample": {"production_A": round(e_a / n, 2), "counting_B": round(e_b / n, 2)},
            "lane_utilization": {"production_A": round(lu_a, 4), "counting_B": round(lu_b, 4),
                                 "one_lane_C": round(rc["SQ_THREAD_CYCLES_VALU"] / (64.0 * rc["SQ_ACTIVE_INST_VALU"]), 5)},
            "model_one_lane_lane_ops_per_sample": round(one / n, 2),
            "model_over_pmc_counting": round(one / e_b, 4),
            "counting_increments_per_sample": round(inc / n, 2),
            "production_over_counting_wave_instructions": round(ra["SQ_INSTS_VALU"] / rb["SQ_INSTS_VALU"], 4),
            "model_production_per_sample": round(one * ra["SQ_INSTS_VALU"] / rb["SQ_INSTS_VALU"] / n, 2),
            "model_over_pmc_production": round(one * ra["SQ_INSTS_VALU"] / rb["SQ_INSTS_VALU"] / e_a, 4),
            "wave_instructions_per_sample": {"production_A": round(ra["SQ_INSTS_VALU"] / n, 3)},
            "algorithmic_lane_ops_per_sample": round(alg_r / n, 2),
            "algorithmic_share_of_executed": round(alg_r / e_a, 4),
        },
        "warmup": {
            "pmc_executed_lane_ops_per_sample": round(e_w / n, 2),
            "lane_utilization": round(lu_w, 4),
            "model_isa_lane_ops_per_sample": round(warm_model / n, 2),
            "model_over_pmc": round(warm_model / e_w, 4),
            "lens_iterations_per_sample": round(lens_iters / n, 4),
            "kernel": "yk_mt_warmup_defer" if defer else "yk_mt_warmup<true, false>",
            "algorithmic_lane_ops_per_sample": round(alg_w / n, 2),
            "algorithmic_share_of_executed": round(alg_w / e_w, 4),
            "calls_consistent": round(executed(wb)[0] / e_w, 4),
        },
    }
    for k in ("SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64", "SQ_INSTS_VALU_CVT", "SQ_INSTS_VALU_ADD_F64",
              "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64", "SQ_INSTS_VALU_FMA_F32"):
        if k in ra:
            res["render"].setdefault("wave_instructions_per_sample_by_type", {})[k] = round(ra[k] / n, 3)
        if k in wa:
            res["warmup"].setdefault("wave_instructions_per_sample_by_type", {})[k] = round(wa[k] / n, 3)
    js = json.dumps(res, indent=1)
    open(out, "w").write(js + "\n")
    print(js)


if __name__ == "__main__":
    main()
