"""FP64 flop models of the render kernel (yk_render_persistent), DESIGN.md §5.

Two models over the kernel's own work counters (a YK_FLAG_COUNT_WORK launch, `Renderer.stats()`):

* ALGORITHMIC — the flops of the reference's own expressions for the work the kernel did
  (sphere.hpp:25-48, math.hpp:10-19, material.hpp, camera.hpp, raytracer.hpp), one flop per
  IEEE add / mul / divide.  This is the roofline's numerator (bench.py `roofline`).
* IMPLEMENTATION — the FP64 operations the gfx950 kernel actually issues for the same work,
  weighted as the hardware counter SQ_INSTS_VALU_FLOPS_FP64 weighs them (v_add/v_mul/
  v_rcp/v_rsq_f64 = 1, v_fma/v_div_fmas_f64 = 2; v_cmp/v_max/v_cvt/v_ldexp/v_div_scale/
  v_div_fixup_f64 = 0 — calibrated on tools/flopcal.hip, profiles/r02_fp64_reconcile.json).
  A division is the refined-reciprocal sequence (rcp + 4 FMA) plus mul + 2 FMA; math::sqrt
  starts at a refined rsq and iterates divisions; the BVH's root bounds add work the reference
  does not have.  Per-unit weights are read off the compiled sequences (yk_device.hpp functions
  compiled alone and counted in the ISA, tools/fp64_reconcile_summary.py).

The counter counts once per WAVE-instruction whatever the exec mask: a launch with all lanes
active reports issued lane-slots / 64; a YK_FLAG_ONE_LANE launch reports exactly the operations
its lanes executed, which is what the implementation model predicts.
"""
from __future__ import annotations

import json
import os

# --- the roofline's peak ---------------------------------------------------------------------
# The FP64 VALU peak is MEASURED, not the datasheet's: tools/ubench.hip times whole launches of
# pure v_fma_f64 streams (8 independent chains per lane, 1-8 waves per SIMD on every SIMD of the
# chip) with HIP events, and the best rate is the peak (profiles/<tag>_ubench.jsonl).  The
# datasheet's MI355X FP64 vector figure is kept beside it for reference.
SPEC_FP64_VALU_TFLOPS = 78.6
UBENCH_EVIDENCE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                               "profiles", "r03_ubench.jsonl")


def ubench_rows(path: str = UBENCH_EVIDENCE):
    with open(path) as f:
        return [json.loads(line) for line in f if line.strip()]


def fp64_valu_peak(path: str = UBENCH_EVIDENCE):
    """(peak TFLOP/s, evidence dict): the best chip-level v_fma_f64 rate in the ubench file, or
    the datasheet figure (said so in the evidence) when the file is absent."""
    if not os.path.exists(path):
        return SPEC_FP64_VALU_TFLOPS, {
            "source": "datasheet (MI355X FP64 vector)",
            "note": f"{os.path.basename(path)} absent: the measured peak (tools/ubench.hip) is unavailable, "
                    "so frac divides by the datasheet figure, like frac_of_spec",
            "spec_fp64_vector_tflops": SPEC_FP64_VALU_TFLOPS}
    rows = ubench_rows(path)
    fma = [r for r in rows if r.get("chip_op") == "fma_f64"]
    if not fma:
        raise ValueError(f"{path}: no chip-level fma_f64 rows")
    best = max(fma, key=lambda r: r["tflops"])
    f32 = [r for r in rows if r.get("chip_op") == "fma_f32"]
    pk = [r for r in rows if r.get("chip_op") == "pk_fma_f32"]
    ev = {
        "source": os.path.relpath(path, os.path.dirname(os.path.dirname(path))),
        "method": "tools/ubench.hip: whole launches of v_fma_f64 (8 independent chains per lane) on "
                  "every SIMD, HIP-event timed, best of 1/2/4/8 waves per SIMD",
        "fma_f64_tflops_by_waves_per_simd": {str(r["waves_per_simd"]): r["tflops"] for r in fma},
        "fma_f64_simd_cycles_per_instr_at_2400mhz": best["simd_cycles_per_instr_at_2400mhz"],
        "fma_f32_best_tflops": max((r["tflops"] for r in f32), default=None),
        "pk_fma_f32_best_tflops": max((r["tflops"] for r in pk), default=None),
        "spec_fp64_vector_tflops": SPEC_FP64_VALU_TFLOPS,
    }
    return best["tflops"], ev

# --- algorithmic (reference expressions) -------------------------------------------------
ALG_PER_SPHERE_TEST = 17  # sphere.hpp:29-33: oc (3), dot (5), len2 - r^2 (6), hb^2 - a*c (3)
ALG_PER_ROOT = 4          # sphere.hpp:36-39: (-hb -/+ sq) / a, one or two roots
ALG_PER_NEWTON_CALL = 1   # math.hpp:12: x = s / 2
ALG_PER_NEWTON_ITER = 3   # math.hpp:14-17: s/x, x + ., ./2
ALG_PER_SEGMENT = 40      # |d|^2, hit record (p, normal, face: 17), normalize (8), scatter (~10)
ALG_PER_SAMPLE = 30       # jitter + camera ray (24), accumulate + attenuation products (~6)


def algorithmic(st: dict) -> float:
    """FP64 flops of the reference's arithmetic for the counted work (per call)."""
    return (st["sphere_tests"] * ALG_PER_SPHERE_TEST + st["sqrt_calls"] * ALG_PER_ROOT
            + st["newton_calls"] * ALG_PER_NEWTON_CALL + st["newton_iters"] * ALG_PER_NEWTON_ITER
            + st["segments"] * ALG_PER_SEGMENT + st["samples"] * ALG_PER_SAMPLE)


def algorithmic_terms() -> str:
    return (f"{ALG_PER_SPHERE_TEST}/sphere test + {ALG_PER_ROOT}/exact root + math::sqrt "
            f"({ALG_PER_NEWTON_CALL}/call + {ALG_PER_NEWTON_ITER}/iteration) + {ALG_PER_SEGMENT}/segment "
            f"+ {ALG_PER_SAMPLE}/sample")


# --- implementation (counter-weighted FP64 operations the kernel issues per lane) ----------
IMPL = {
    # leaf: the reference's discriminant (9 add + 8 mul, no contraction)
    "sphere_test": 17,
    # disc >= 0: sqrt_bound (rsq + 2 mul + 2 fma = 7), two roots x 1/a (4), margin (4),
    # r2 + m, r1 - m, and the upper bound (2)
    "leaf_disc_pos": 19,
    # exact candidate: discriminant again (17) + (-hb - sq) + div_by (mul + 2 fma = 5); the
    # second root (another 6) when the first is below t_min is folded into the 1.1 factor
    "candidate": 17 + 6 * 1.1,
    "newton_call": 17,   # sqrt_start: rsq, 2 mul, 7 fma
    "newton_iter": 16,   # rcp_refined (rcp + 4 fma = 9) + div_pos (5) + add + mul 0.5
    # every segment: a = len2(d) (5) + rcp_bound (rcp + 2 fma = 5); the shading length (len2 5)
    # and divs_fast (rcp_refined 9 + 3 x div_by 5 = 24) of the one shared normalisation
    "segment": 10 + 29,
    # a hit: p = o + d T (6), p - c (3), divs_fast by the radius (24), dot(d, n) (5)
    "hit": 38,
    "lambertian": 9 + 3,          # random_vec (3 x 3 adds; the powers of two are v_ldexp) + add
    "metal": 12 + 5,              # reflect (6 mul + 6 add) + dot(nd, n)
    # fuzz: random_vec (9) + len2 (5) + divs_fast (24) + uniform (3) + 2 scalings (6) + add (3)
    "metal_fuzz": 50,
    # dielectric (yk_device.hpp reflectance etc.): half the hits divide 1/ior (14); dot, 1-ct^2,
    # ratio*sn (8); Schlick (25); uniform (2); reflect (12) or refract (21): ~58
    "dielectric": 58,
    "sky": 8,                     # (y + 1)/2 and the lerp (5 add + 3 mul)
    "attenuation": 3,             # unwinding: 3 mul per scattering sphere on the stack
    # sample start: 2 uniform(0,1) (2 each) + 2 Markstein quotients (add + mul + 2 fma = 6 each)
    # + camera ray (5 x 3)
    "sample": 31,
    "candidate_rcp": 9,           # rcp_refined(a), once per segment with candidates (~ hits)
}


def implementation(st: dict) -> float:
    """Counter-weighted FP64 operations the kernel executes for the counted work (per call)."""
    w = st["work"]
    dpos, lamb, metal, fuzz, diel = w[0], w[1], w[2], w[3], w[4]
    hits = lamb + metal + diel
    sky = st["segments"] - hits  # every other segment that ran shading ended in the sky
    return (st["sphere_tests"] * IMPL["sphere_test"] + dpos * IMPL["leaf_disc_pos"]
            + st["sqrt_calls"] * IMPL["candidate"] + hits * IMPL["candidate_rcp"]
            + st["newton_calls"] * IMPL["newton_call"] + st["newton_iters"] * IMPL["newton_iter"]
            + st["segments"] * IMPL["segment"] + hits * IMPL["hit"]
            + lamb * IMPL["lambertian"] + metal * IMPL["metal"] + fuzz * IMPL["metal_fuzz"]
            + diel * IMPL["dielectric"] + sky * IMPL["sky"] + (lamb + metal) * IMPL["attenuation"]
            + st["samples"] * IMPL["sample"])


# --- the VALU lane-op roofline: the path's whole work -----------
# SURVEY §8(d) counts, beside the FP64 flops, the RNG's integer work.  ALGORITHMIC lane-ops are the
# reference's own operators for the work done, one per C++ operator (an IEEE add / mul / divide /
# conversion / compare, a 32-bit shift / xor / and / or / multiply / add), per lane:
#   * the FP64 flops above (algorithmic(st));
#   * mt19937 (random.hpp:43-151).  A sample's engine is seeded from its seed (x_i =
#     1812433253 (x_{i-1} ^ x_{i-1} >> 30) + i, :69-81: >>, ^, *, + = 4 ops per step) and output j
#     (j < 227) is temper(x_{j+397} ^ mix(x_j, x_{j+1})) (:114-131, :95-105).  The least work that
#     yields the draws a sample makes: the walk to x_397 (397 steps) once, then per draw the next
#     x_{j+397} (one step), the twisted word (mix: (a & U) | (b & L), >> 1, the odd select, two
#     xors: 7) and the tempering (4 shifts, 2 ands, 4 xors: 10): 21 integer ops per word; plus
#     generate_canonical's FP64 part per word (the u32 -> double conversion; per canonical of two
#     words u0 + u1 2^32 (mul, add), / 2^64, >= 1: 3 ops per word).  A sample past draw 227 has
#     its full engine seeded (623 steps) and twisted (624 words x 7 ops per twist, work[7]).
#   * xor128 (random.hpp:18-41): 7 integer ops per word (<<, ^, >>, ^, >>, ^, ^), no seeding.
# Classes, because the VALU issues them at different rates (tools/ubench.hip, 8 waves per SIMD):
# FP64 (v_fma_f64's cost: ~4.4 SIMD cycles per wave-instruction), 32-bit multiplies
# (v_mul_lo_u32, ~4.4), other 32-bit integer ops (v_xor_b32, ~2.5).  The PEAK of a mix is the
# rate at which every SIMD would issue exactly that mix with all 64 lanes of every instruction
# active: 64 x 1024 SIMDs x 2.4 GHz x N_total / sum_k N_k c_k.
SEED_STEP_OPS = 4
SEED_STEP_MULS = 1
WALK_STEPS = 397
DRAW_INT_OPS = 21       # one seeding step (4, one multiply) + the twisted word (7) + tempering (10)
DRAW_MULS = 1
WORD_F64_OPS = 3        # generate_canonical's conversion and arithmetic, per word
TWIST_WORD_OPS = 7
MT_STATE_WORDS = 624
X128_WORD_OPS = 7
CAMERA_F64_OPS = 24     # the start's jitter + camera ray (part of ALG_PER_SAMPLE, done by the warm-up)
UBENCH_R05 = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                          "profiles", "r05_ubench.jsonl")


UBENCH_R03D = os.path.join(os.path.dirname(UBENCH_EVIDENCE), "r03d_ubench.jsonl")


def issue_costs(path: str = UBENCH_R05, fallback: str = UBENCH_R03D):
    """SIMD cycles per wave64 instruction at 2.4 GHz of each op class, at the saturating 8 waves
    per SIMD (tools/ubench.hip chip rows): {'f64', 'mul32', 'int32'} and the evidence file."""
    src = path if os.path.exists(path) else fallback
    rows = [r for r in ubench_rows(src) if r.get("waves_per_simd") == 8 and "chip_op" in r]
    by = {r["chip_op"]: r["simd_cycles_per_instr_at_2400mhz"] for r in rows}
    int32 = by.get("xor_b32", by["xor_shr_u32"] / 2)  # xor_shr_u32 issues two instructions
    return {"f64": by["fma_f64"], "mul32": by["mul_lo_u32"], "int32": int32}, os.path.relpath(
        src, os.path.dirname(os.path.dirname(src)))


def lane_ops(st: dict, engine: str = "mt19937") -> dict:
    """Algorithmic lane-ops of one counted call by class and by kernel (the seed-walk kernel
    yk_mt_warmup: the walk, the start's draws and camera ray; the render: the rest)."""
    n = st["samples"]
    w = st["work"]
    words, swords, twists, fb = w[5], w[6], w[7], st["mt_fallbacks"]
    f64_all = algorithmic(st) + WORD_F64_OPS * words
    if engine == "xor128":  # no warm-up kernel: the render does the whole start
        warm = {"f64": 0.0, "mul32": 0.0, "int32": 0.0}
        rend = {"f64": f64_all, "mul32": 0.0, "int32": X128_WORD_OPS * words}
        return {"warmup": warm, "render": rend}
    walk_int = n * WALK_STEPS * (SEED_STEP_OPS - SEED_STEP_MULS)
    warm = {"f64": n * CAMERA_F64_OPS + WORD_F64_OPS * swords,
            "mul32": n * WALK_STEPS * SEED_STEP_MULS + swords * DRAW_MULS,
            "int32": walk_int + swords * (DRAW_INT_OPS - DRAW_MULS)}
    rw = words - swords
    rend = {"f64": f64_all - warm["f64"],
            "mul32": rw * DRAW_MULS + fb * (MT_STATE_WORDS - 1) * SEED_STEP_MULS,
            "int32": rw * (DRAW_INT_OPS - DRAW_MULS) + fb * (MT_STATE_WORDS - 1) * (SEED_STEP_OPS - SEED_STEP_MULS)
                     + twists * MT_STATE_WORDS * TWIST_WORD_OPS}
    return {"warmup": warm, "render": rend}


def mix_peak(mix: dict, costs: dict, simds: int = 1024, ghz: float = 2.4) -> float:
    """Lane-ops/s at which the chip issues this mix with every lane of every instruction active."""
    tot = sum(mix.values())
    cyc = sum(mix[k] * costs[k] for k in mix) / 64.0  # SIMD cycles for the mix
    return tot / cyc * simds * ghz * 1e9 if cyc else 0.0


def lane_op_roofline(ops: dict, seconds: float, costs: dict) -> dict:
    tot = sum(ops.values())
    peak = mix_peak(ops, costs)
    ach = tot / seconds if seconds > 0 else 0.0
    return {"algorithmic": round(tot), "achieved": round(ach / 1e12, 4), "peak": round(peak / 1e12, 4),
            "unit": "T lane-ops/s", "frac": round(ach / peak, 5) if peak else None,
            "mix": {k: round(v / tot, 4) if tot else 0.0 for k, v in ops.items()}}
