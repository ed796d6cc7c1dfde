"""The bench line's roofline recomputes from the committed evidence (CPU; profiles/).

* the FP64 implementation model (uecraytracing_amd/flops.py) agrees with the hardware counter
  read on a one-lane-per-wave launch (profiles/r02_fp64_reconcile.json) within 1.5x;
* the latest committed bench line: launches x launch_ms <= ms_per_step (the per-launch duration
  counts overlapping spans once), `achieved` = algorithmic flops per launch / launch_ms, and the
  rocprofv3 kernel trace of the same build gives the same per-launch duration within 5%.
"""
import glob
import json
import os

import pytest

from uecraytracing_amd import flops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")


def latest_bench():
    """The bench line of the build profiles/pmc_summary.json was collected for (collect_profiles.sh
    installs both from one run), else the newest tag: r02 < r02a..r02z < r02aa.. (a plain sort
    would put r02q after r02bo)."""
    try:
        src = json.load(open(os.path.join(PROF, "pmc_summary.json")))["source"]
        tag = src.split("/")[1]
        f = os.path.join(PROF, f"{tag}_bench.json")
        if os.path.exists(f):
            return f
    except (OSError, KeyError, IndexError, ValueError):
        pass
    files = glob.glob(os.path.join(PROF, "r0*_bench.json"))
    if not files:
        pytest.skip("no bench line in profiles/")

    def key(f):
        tag = os.path.basename(f)[: -len("_bench.json")]
        rnd, letters = tag[:3], tag[3:].lstrip("_")
        return (rnd, len(letters), letters)
    return max(files, key=key)


def test_fp64_counter_reconciles_with_the_implementation_model():
    rec = json.load(open(os.path.join(PROF, "r02_fp64_reconcile.json")))
    st = rec["work"]
    impl = flops.implementation(st)
    counter = rec["executed_fp64_one_lane_counter"]
    assert 1 / 1.5 < impl / counter < 1.5
    # the algorithmic model is a subset of what executes; lane-slots issued bound it from above
    assert flops.algorithmic(st) < counter < rec["issued_lane_slots_fp64"]
    # the calibration found the counter per wave-instruction, independent of the exec mask
    fma = [c for c in rec["calibration"]["cases"] if c["op"] == "fma_f64"]
    assert {c["active_lanes"] for c in fma} == {64, 16}
    assert all(abs(c["flops_fp64_per_wave_instr"] - 2.0) < 0.01 for c in fma)


def test_fp64_peak_is_the_measured_fma_rate():
    """profiles/r03_ubench.jsonl (tools/ubench.hip, HIP-event timed launches of pure v_fma_f64 on
    every SIMD): the peak is its best rate; at 8 waves per SIMD the FP64 FMA costs what the packed
    FP32 FMA costs (~4 SIMD cycles per wave-instruction at 2.4 GHz), about twice the plain FP32
    FMA — the datasheet's 78.6 TF (FP64 = half the FP32 vector peak) holds, and the measured rate
    sits within 15% below it (the clock under load)."""
    peak, ev = flops.fp64_valu_peak()
    rows = flops.ubench_rows()
    fma64 = [r for r in rows if r.get("chip_op") == "fma_f64"]
    assert peak == max(r["tflops"] for r in fma64)
    assert 0.85 * flops.SPEC_FP64_VALU_TFLOPS <= peak <= flops.SPEC_FP64_VALU_TFLOPS
    best = max(fma64, key=lambda r: r["tflops"])
    assert 3.6 <= best["simd_cycles_per_instr_at_2400mhz"] <= 4.8
    pk = max((r for r in rows if r.get("chip_op") == "pk_fma_f32"), key=lambda r: r["tflops"])
    f32 = max((r for r in rows if r.get("chip_op") == "fma_f32"), key=lambda r: r["tflops"])
    assert abs(pk["simd_cycles_per_instr_at_2400mhz"] / best["simd_cycles_per_instr_at_2400mhz"] - 1) < 0.1
    assert f32["tflops"] > 1.4 * peak
    # each op's rate rises with waves per SIMD up to the best one (a saturating issue rate)
    by = sorted(fma64, key=lambda r: r["waves_per_simd"])
    assert all(a["tflops"] <= b["tflops"] * 1.02 for a, b in zip(by, by[1:]))


def test_bench_roofline_is_admissible():
    b = json.load(open(latest_bench()))
    rf = b["roofline"]
    assert rf["bound"] == "valu"
    if "peak_evidence" in rf:  # round 3 on: the measured peak of profiles/r03_ubench.jsonl
        assert rf["peak"] == flops.fp64_valu_peak()[0]
    assert rf["launches_per_step"] * rf["launch_ms"] <= b["ms_per_step"] * 1.001
    ach = rf["algorithmic_flops_per_launch"] / (rf["launch_ms"] * 1e-3) / 1e12
    assert abs(ach - rf["achieved"]) / rf["achieved"] < 0.01
    assert abs(rf["achieved"] / rf["peak"] - rf["frac"]) / rf["frac"] < 0.01


def test_rocprof_union_agrees_with_bench_launch_ms():
    bench = latest_bench()
    tag = os.path.basename(bench)[: -len("_bench.json")]
    union = os.path.join(PROF, f"{tag}_kernel_union.json")
    if not os.path.exists(union):
        pytest.skip("no kernel trace union for the latest bench")
    b = json.load(open(bench))
    u = json.load(open(union))
    # round 4 on, the traced run mixes synced calls (launches of 4-32 spp) and back-to-back ones:
    # compare per 32-spp launch equivalent (tools/kernel_union.py)
    # (round 6 on: the traced run is 2 warm-up + 6 timed steps, six of its eight calls in flight
    # like the bench's; union_last_call_per_launch_ms, the last call alone, includes its lone drain)
    per = u.get("union_per_launch_equiv_ms", u["union_per_dispatch_ms"])
    assert abs(per - b["roofline"]["launch_ms"]) / b["roofline"]["launch_ms"] < 0.05


def test_peak_falls_back_to_the_datasheet_without_the_ubench_file(tmp_path):
    """No ubench evidence (a tree without profiles/): the datasheet figure, said so."""
    peak, ev = flops.fp64_valu_peak(str(tmp_path / "absent.jsonl"))
    assert peak == flops.SPEC_FP64_VALU_TFLOPS
    assert "datasheet" in ev["source"] and "absent" in ev["note"]


def test_lane_op_model_counts_the_rng_work():
    """SURVEY §8(d)'s algorithmic work includes the RNG's integer ops: the
    seed walk (397 steps of 4 ops per sample) dominates a sample's lane-ops, the per-word ops
    follow the words drawn, and the warm-up / render split adds up to the whole."""
    st = {"samples": 1000, "segments": 2100, "sphere_tests": 4000, "sqrt_calls": 1300, "newton_calls": 3000,
          "newton_iters": 3000, "mt_fallbacks": 0, "work": [2000, 900, 300, 100, 200, 11000, 4400, 0]}
    lo = flops.lane_ops(st)
    walk = st["samples"] * flops.WALK_STEPS * flops.SEED_STEP_OPS
    assert lo["warmup"]["mul32"] + lo["warmup"]["int32"] == walk + st["work"][6] * flops.DRAW_INT_OPS
    assert lo["render"]["mul32"] + lo["render"]["int32"] == (st["work"][5] - st["work"][6]) * flops.DRAW_INT_OPS
    f64 = flops.algorithmic(st) + flops.WORD_F64_OPS * st["work"][5]
    assert abs(lo["warmup"]["f64"] + lo["render"]["f64"] - f64) < 1e-6
    # the integer work outweighs the FP64 work per sample, as the verdict estimated
    tot = {k: lo["warmup"][k] + lo["render"][k] for k in lo["render"]}
    assert tot["mul32"] + tot["int32"] > 4 * tot["f64"]
    # a mix's peak lies between its classes' peaks; all-FP64 is the v_fma_f64 instruction rate
    costs, _ = flops.issue_costs()
    p64 = flops.mix_peak({"f64": 1.0, "mul32": 0.0, "int32": 0.0}, costs)
    assert abs(p64 - 64 * 1024 * 2.4e9 / costs["f64"]) / p64 < 1e-9
    pint = flops.mix_peak({"f64": 0.0, "mul32": 0.0, "int32": 1.0}, costs)
    assert p64 < flops.mix_peak(tot, costs) < pint


def test_issue_costs_are_measured_rates():
    """profiles/r05_ubench.jsonl (tools/ubench.hip at 8 waves per SIMD): a plain 32-bit op issues
    at ~2.5 SIMD cycles per wave-instruction, the 32-bit multiply and the FP64 FMA at ~4.4, and the
    seed walk's step (shift, xor, 64-bit multiply-add) costs their sum."""
    costs, src = flops.issue_costs()
    assert "r05_ubench" in src
    assert 2.0 < costs["int32"] < 3.0 and 3.8 < costs["mul32"] < 5.0 and 3.8 < costs["f64"] < 5.0
    rows = {r["chip_op"]: r for r in flops.ubench_rows(flops.UBENCH_R05)
            if r.get("waves_per_simd") == 8 and "chip_op" in r}
    walk = rows["walk_step"]["simd_cycles_per_instr_at_2400mhz"]
    parts = 2 * rows["xor_b32"]["simd_cycles_per_instr_at_2400mhz"] + rows["mad_u64_u32"]["simd_cycles_per_instr_at_2400mhz"]
    assert abs(walk / parts - 1) < 0.1


def test_lane_op_reconciliation_with_the_pmc_counters():
    """profiles/pmc_lane_ops.json (tools/gpu_lane_ops.sh): the render's executed lane-ops from
    the one-lane count agree with the PMC-derived ones (SQ_INSTS_VALU x 64 x lane utilisation) of
    the same binary within 10%, and of the production instance within 10% once the counting
    instance's wave-instruction ratio carries it over; the warm-up's ISA model agrees with its PMC figure
    within 10%; the algorithmic lane-ops are a part of what executes."""
    f = os.path.join(PROF, "pmc_lane_ops.json")
    if not os.path.exists(f):
        pytest.skip("no lane-op reconciliation in profiles/")
    rec = json.load(open(f))
    r, w = rec["render"], rec["warmup"]
    assert rec["images_equal"]
    assert abs(r["model_over_pmc_counting"] - 1) < 0.10
    assert abs(r["model_over_pmc_production"] - 1) < 0.10
    assert abs(w["model_over_pmc"] - 1) < 0.10
    assert r["lane_utilization"]["one_lane_C"] < 1.5 / 64 < 0.3 < r["lane_utilization"]["production_A"]
    assert 0 < r["algorithmic_share_of_executed"] < 1 and 0 < w["algorithmic_share_of_executed"] < 1.5


def test_bench_line_carries_the_lane_op_roofline():
    b = json.load(open(latest_bench()))
    vo = b["roofline"].get("valu_ops")
    if vo is None:
        pytest.skip("bench line from before the lane-op roofline")
    for k in ("render", "warmup", "step"):
        x = vo[k]
        assert set(("algorithmic", "achieved", "peak", "frac")) <= set(x)
        assert 0 < x["frac"] < 1
        assert abs(x["achieved"] / x["peak"] - x["frac"]) / x["frac"] < 0.01
    # the step's work is both kernels' work
    per_step = vo["render"]["algorithmic"] * b["roofline"]["launches_per_step"] + \
        vo["warmup"]["algorithmic"] * b["roofline"]["launches_per_step"]
    assert abs(per_step / vo["step"]["algorithmic"] - 1) < 0.01
    h = b["roofline"]["hbm"]
    tps = h.get("render_kernel_traffic_per_sample", h.get("traffic_per_sample"))
    if tps:
        r = h.get("render_kernel_traffic_over_algorithmic", h.get("traffic_over_algorithmic"))
        assert abs(tps / h["algorithmic_bytes_per_sample"] / r - 1) < 0.01


def test_measured_hbm_covers_every_kernel_of_the_step():
    """profiles/pmc_hbm.json (tools/pmc_hbm.py): the render kernel's bytes per
    sample are the render summary's of the same PMC run, the step's figure is the sum over render,
    warm-up and reduce, and the bench line's `hbm.measured` recomputes from it: bytes per sample x
    the step's samples / ms_per_step, its fractions of the 8 TB/s spec and the 6.29 TB/s measured
    copy rate."""
    import bench
    f = os.path.join(PROF, "pmc_hbm.json")
    if not os.path.exists(f):
        pytest.skip("no per-kernel HBM summary in profiles/")
    rec = json.load(open(f))
    ks = rec["kernels"]
    assert set(ks) == {"render", "warmup", "reduce"}
    assert abs(sum(k["bytes_per_sample"] for k in ks.values()) - rec["bytes_per_sample"]) < 1e-6
    tag = rec["source"].split("gpurun_out/")[1].split("/")[0]
    summ = os.path.join(PROF, f"{tag}_pmc_summary.json")
    if os.path.exists(summ):
        r = json.load(open(summ))["hbm_bytes_per_sample"]
        assert abs(ks["render"]["bytes_per_sample"] / r - 1) < 1e-3
    # a launch's scratch round trip: the warm-up writes each sample's 64-B start record, the
    # render reads it and writes a 32-B colour record, the reduce reads that
    assert ks["warmup"]["write_bytes_per_sample"] > 64 and ks["render"]["fetch_bytes_per_sample"] > 64
    assert ks["render"]["write_bytes_per_sample"] > 32 and ks["reduce"]["fetch_bytes_per_sample"] > 32
    m = bench.hbm_measured(1000, 2.0, 0.5, f)
    assert abs(m["achieved"] - rec["bytes_per_sample"] * 1000 / 2e-3 / 1e9) < 0.01
    assert abs(m["frac"] - m["achieved"] / bench.HBM_PEAK_GBPS) < 1e-4
    assert abs(m["frac_of_measured"] - m["achieved"] / bench.HBM_MEASURED_GBPS) < 1e-4
    b = json.load(open(latest_bench()))
    bm = b["roofline"]["hbm"].get("measured")
    if bm:
        spp = b["config"]["spp"]
        W, H = (int(x) for x in b["config"]["image"].split("x"))
        want = bm["bytes_per_sample"] * W * H * spp / b["n_gpus"] / (b["ms_per_step"] * 1e-3) / 1e9
        assert abs(bm["achieved"] / want - 1) < 0.01
        assert 0 < bm["frac"] < 1
