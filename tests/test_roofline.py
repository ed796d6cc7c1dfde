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
    per = u.get("union_per_launch_equiv_ms", u["union_per_dispatch_ms"])
    assert abs(per - b["roofline"]["launch_ms"]) / b["roofline"]["launch_ms"] < 0.05


def test_peak_falls_back_to_the_datasheet_without_the_ubench_file(tmp_path):
    """No ubench evidence (a tree without profiles/): the datasheet figure, said so."""
    peak, ev = flops.fp64_valu_peak(str(tmp_path / "absent.jsonl"))
    assert peak == flops.SPEC_FP64_VALU_TFLOPS
    assert "datasheet" in ev["source"] and "absent" in ev["note"]
