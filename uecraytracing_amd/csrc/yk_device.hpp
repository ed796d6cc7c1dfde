// yk_device.hpp — per-lane arithmetic of one sample, gfx950 device code.
//
// Every function reproduces the reference's IEEE-double evaluation order operation for
// operation (the file is compiled with -ffp-contract=off: no FMA contraction), so a sample's
// colour is bit-identical to yk::raytracer<double,double>::ray_color.  Citations are
// /root/reference/<file>:<line>.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ykd {

// ------------------------------------------------------------------------------------------
// vec3 (yk/vec3.hpp) — only the operations the hot path uses, same association order.
struct v3 {
  double x, y, z;
};
__device__ __forceinline__ v3 add(v3 a, v3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ v3 sub(v3 a, v3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ v3 mul(v3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ v3 divs(v3 a, double s) { return {a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ v3 neg(v3 a) { return {-a.x, -a.y, -a.z}; }
// dot(): vec3.hpp:145-147 → (x*x' + y*y') + z*z'
__device__ __forceinline__ double dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
// length_squared(): vec3.hpp:129
__device__ __forceinline__ double len2(v3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }

// math::sqrt (math.hpp:10-19): x = s/2, then x = (x + s/x)/2 until two iterates are equal.
// Not IEEE sqrt (differs by an ulp on ~25% of inputs), so its RESULT is reproduced exactly --
// but not its path.  The loop can only stop at a fixed point of g(x) = fl(fl(x + fl(s/x))/2),
// and for normal s that fixed point is UNIQUE: in units of ulp(x), x is fixed iff
// RN(2(sqrt(s) - x)) is 0, or +-1 with x's significand even, which at most one double satisfies
// ("math::sqrt").  So the same iteration started at the IEEE sqrt (within half an
// ulp) ends at the reference's value after 1-2 steps instead of 5-17.  Checked against the
// reference loop on every s = 2^k +- m ulp (k = -1074..1023, m < 2e5: 8.4e8 values) and 3e7
// random values: only the smallest subnormal differs (s/2 underflows to 0), hence the guard
// below, under which the reference start is kept.  The iteration bound only matters for NaN/inf.
// ---- division and square roots without the special-case steps ------------------------------
// A correctly rounded double division on gfx950 is the compiler's sequence
//   div_scale(d), div_scale(n), rcp, 4 fma (reciprocal refinement), mul, fma (residual),
//   div_fmas, div_fixup                          (measured 49 cycles/SIMD per wave, tools/ubench)
// div_scale only rescales operands at the extremes of the exponent range, div_fmas is a plain
// fma when nothing was scaled, and div_fixup only rewrites NaN/inf/zero/denormal cases.  For
// operands in [2^-400, 2^400] (or a zero numerator) the sequence below is therefore the same
// arithmetic, operation for operation, minus those steps -- and the refined reciprocal depends
// only on the divisor, so it is computed once for a vector / scalar.  Bit-identical to `/`:
// checked by tests/test_gpu_parity.py::test_fast_division_is_ieee_division (ykgpu_math_div).
__device__ __forceinline__ bool div_range(double x) { return fabs(x) >= 0x1p-400 && fabs(x) <= 0x1p400; }
__device__ __forceinline__ bool num_range(double x) { return x == 0.0 || div_range(x); }
__device__ __forceinline__ double rcp_refined(double s) {
  const double r0 = __builtin_amdgcn_rcp(s);
  double t = __builtin_fma(-s, r0, 1.0);
  const double r1 = __builtin_fma(r0, t, r0);
  t = __builtin_fma(-s, r1, 1.0);
  return __builtin_fma(r1, t, r1);
}
// n / s given r = rcp_refined(s), both in range.  A zero numerator's quotient is q0 = n * r with
// the IEEE sign; the final fma would turn -0 into +0, and for n != 0 q and q0 share their sign,
// so copysign(q, q0) is exact in both cases (one v_bfi).
__device__ __forceinline__ double div_by(double n, double s, double r) {
  const double q0 = n * r;
  const double e = __builtin_fma(-s, q0, n);
  return __builtin_copysign(__builtin_fma(e, r, q0), q0);
}
// Same for n > 0 (math::sqrt's s / x).
__device__ __forceinline__ double div_pos(double n, double s, double r) {
  const double q0 = n * r;
  return __builtin_fma(__builtin_fma(-s, q0, n), r, q0);
}
// vector / scalar: fast quotients for every lane; if any lane of the wave has an operand outside
// the range, the whole wave recomputes with the full division (same bits for in-range lanes), so
// there is no per-lane branch nest.
__device__ __forceinline__ v3 divs_fast(v3 a, double s) {
  const double r = rcp_refined(s);
  v3 q = {div_by(a.x, s, r), div_by(a.y, s, r), div_by(a.z, s, r)};
  const bool ok = div_range(s) && num_range(a.x) && num_range(a.y) && num_range(a.z);
  if (__builtin_expect(__ballot(!ok) != 0, 0)) q = divs(a, s);
  return q;
}
// the same with the divisor's refined reciprocal r = rcp_refined(s) computed beforehand (the hit
// normal's division by the radius: yk_mat_prep computes it once per sphere)
__device__ __forceinline__ v3 divs_fast_r(v3 a, double s, double r) {
  v3 q = {div_by(a.x, s, r), div_by(a.y, s, r), div_by(a.z, s, r)};
  const bool ok = div_range(s) && num_range(a.x) && num_range(a.y) && num_range(a.z);
  if (__builtin_expect(__ballot(!ok) != 0, 0)) q = divs(a, s);
  return q;
}
// n / d for n >= 0 and a small integer d with y = RN(1/d) from the host: Markstein's theorem
// (y correctly rounded, q0 = RN(n*y) within an ulp => fma(fma(-d, q0, n), y, q0) = RN(n/d)).
__device__ __forceinline__ double div_markstein(double n, double d, double y) {
  const double q0 = n * y;
  return __builtin_fma(__builtin_fma(-d, q0, n), y, q0);
}

// Bounds-only approximations (the BVH's root bounds; never a result):
// v_rsq_f64 / v_rcp_f64 are within 2^-23 (ISA: 2^29 ulp; measured 2^-24.2), one Newton step
// squares that: relative error < 2^-44.
__device__ __forceinline__ double sqrt_bound_r(double x, double r) {  // x >= 0, r = rsq(x)
  const double y = x * r, h = 0.5 * r;
  const double y1 = __builtin_fma(__builtin_fma(-y, y, x), h, y);
  return x == 0.0 ? 0.0 : y1;
}
__device__ __forceinline__ double sqrt_bound(double x) { return sqrt_bound_r(x, __builtin_amdgcn_rsq(x)); }
__device__ __forceinline__ double rcp_bound(double a) {  // a > 0
  const double r0 = __builtin_amdgcn_rcp(a);
  return __builtin_fma(r0, __builtin_fma(-a, r0, 1.0), r0);
}
// Start of math::sqrt's loop (any start gives the same fixed point; this one is the library's
// correctly rounded sqrt without its denormal rescaling, valid for s in [2^-400, 2^400]).
__device__ __forceinline__ double sqrt_start_r(double s, double r) {  // r = rsq(s), given
  double g = s * r, h = r * 0.5;
  const double e = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, e, g);
  h = __builtin_fma(h, e, h);
  double d = __builtin_fma(-g, g, s);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, s);
  return __builtin_fma(d, h, g);
}
__device__ __forceinline__ double sqrt_start(double s) { return sqrt_start_r(s, __builtin_amdgcn_rsq(s)); }

__device__ __forceinline__ double nsqrt_impl(double s, uint32_t& iters, const double* rsq = nullptr) {
  double x, prev = 0.0;
  if (s >= 0x1p-400 && s <= 0x1p400) {
    // ONE step from r = RN(sqrt(s)) lands on the loop's fixed point: in ulps of r,
    // fl(s/r) = r + RN(2(sqrt(s) - r)), so g(r) is r or the neighbour that the sum's
    // round-to-even picks, and that neighbour is the fixed point.  Checked against the
    // reference loop on 4.2e8 values (every s = 2^k +- m ulp, |k| <= 400, m < 2e5, and 1e8
    // random) and by tests/test_oracle_golden.py.  (The division needs no special-case steps
    // for iterates within [2^-201, 2^201].)
    x = rsq ? sqrt_start_r(s, *rsq) : sqrt_start(s);  // (rsq: the same v_rsq_f64 of s, computed before)
    ++iters;
    return (x + div_pos(s, x, rcp_refined(x))) / 2.0;
  }
  x = (s >= 0x1p-1000 && s <= 0x1.fffffffffffffp+1023) ? __builtin_sqrt(s) : s / 2.0;
  for (int guard = 0; x != prev && guard < 4096; ++guard) {
    prev = x;
    x = (x + s / x) / 2.0;
    ++iters;
  }
  return x;
}
__device__ __forceinline__ double nsqrt(double s) {
  uint32_t it = 0;
  return nsqrt_impl(s, it);
}

// Same, counting calls and loop iterations (work counters of the roofline model).
__device__ __forceinline__ double nsqrt_c(double s, uint32_t& calls, uint32_t& iters) {
  ++calls;
  return nsqrt_impl(s, iters);
}
__device__ __forceinline__ double nsqrt_c_r(double s, double rsq, uint32_t& calls, uint32_t& iters) {
  ++calls;
  return nsqrt_impl(s, iters, &rsq);
}

__device__ __forceinline__ v3 normalized(v3 a) { return divs(a, nsqrt(len2(a))); }  // :127,132
// reflect(): vec3.hpp:199-202, v - (2*dot(v,n))*n
__device__ __forceinline__ v3 reflect(v3 v, v3 n) { return sub(v, mul(n, 2.0 * dot(v, n))); }
// near_zero(): vec3.hpp:76-80 — tests |x|, |y| and |x| again (z is never tested)
__device__ __forceinline__ bool near_zero(v3 a) {
  const double ax = a.x > 0 ? a.x : -a.x, ay = a.y > 0 ? a.y : -a.y;
  return (ax < 1e-8) && (ay < 1e-8) && (ax < 1e-8);
}

// ------------------------------------------------------------------------------------------
// mt19937 (random.hpp:43-151), one fresh engine per sample (source.cpp:154-158).
//
// A full engine is 624 words; seeding it and twisting it costs ~8 µs per sample on the CPU
// (90% of the reference's time).  A sample draws 11 words on average (p99 58), so the lane
// keeps three CURSORS into the seeding sequence x_i instead of the state:
//   output j (j < 227) = temper( x_{j+397} ^ mix(x_j, x_{j+1}) )      (M_gen_rand, :118-121)
// with x_i = 1812433253*(x_{i-1} ^ x_{i-1}>>30) + i (seed(), :69-81).  Cursor A carries
// (x_j, x_{j+1}), cursor B carries x_{j+397}; each draw steps both by one.  Start-up is the
// 397-step walk of B.  Draw 227 and later need words the first twist already rewrote, so
// the lane then materialises the real 624-word state in its slot of a global scratch buffer
// (same seed, same twist) and continues from index 227 — exact for any number of draws.
constexpr uint32_t kMtN = 624, kMtM = 397, kLazyDraws = kMtN - kMtM;  // 227

__device__ __forceinline__ uint32_t mt_seed_step(uint32_t prev, uint32_t i) {
  return 1812433253u * (prev ^ (prev >> 30)) + i;
}
// gfx950's three-input bitwise op (v_bitop3_b32: bit i of the result is bit
// (a_i << 2 | b_i << 1 | c_i) of the table): a ^ (b & c) is table 0x78, (a & c) | (b & ~c) 0xE4
__device__ __forceinline__ uint32_t xor_and(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x78);
}
__device__ __forceinline__ uint32_t mt_mix(uint32_t hi_src, uint32_t lo_src) {
  // y = upper bit of hi_src, lower 31 of lo_src; (y >> 1) ^ (y odd ? 0x9908b0df : 0), the
  // odd test read from lo_src (y & 1 = lo_src & 1) as an all-ones / zero mask: 5 instructions
  const uint32_t y = __builtin_amdgcn_bitop3_b32(hi_src, lo_src, 0x80000000u, 0xE4);
  const uint32_t odd = 0u - (lo_src & 1u);
  return xor_and(y >> 1, odd, 0x9908b0dfu);
}
__device__ __forceinline__ uint32_t mt_temper(uint32_t z) {  // random.hpp:98-102
  z ^= (z >> 11);
  z = xor_and(z, z << 7, 0x9d2c5680u);   // z ^= (z << 7) & 0x9d2c5680
  z = xor_and(z, z << 15, 0xefc60000u);  // z ^= (z << 15) & 0xefc60000
  z ^= (z >> 18);
  return z;
}

struct MtLane {
  uint32_t a0, a1, b;  // x_j, x_{j+1}, x_{j+397}
  uint32_t j;          // index of the next output
  uint32_t seed;
  uint32_t* state;     // this lane's 624-word scratch (used only once j reaches 227)
};
// A sample used the scratch engine iff it drew more than 227 words.
__device__ __forceinline__ bool mt_used_fallback(const MtLane& g) { return g.j > kLazyDraws; }
// Work counters (YK_FLAG_COUNT_WORK; the VALU lane-op roofline, uecraytracing_amd/flops.py): the
// words a sample's engine has drawn, and the scratch engine's 624-word twists they needed — the
// first at draw 227 (mt_slow), then one per 624 draws (random.hpp:95-105, 114-131).
__device__ __forceinline__ uint32_t rng_words(const MtLane& g) { return g.j; }
__device__ __forceinline__ uint32_t rng_twists(const MtLane& g) { return g.j > kLazyDraws ? 1u + (g.j - 1u) / kMtN : 0u; }

__device__ __forceinline__ void mt_start(MtLane& g, uint32_t seed) {
  g.seed = seed;
  g.j = 0;
  g.a0 = seed;
  uint32_t x = mt_seed_step(seed, 1);
  g.a1 = x;
#pragma unroll 8
  for (uint32_t i = 2; i <= kMtM; ++i) x = mt_seed_step(x, i);
  g.b = x;
}

// Start from a precomputed x_397 (yk_mt_warmup kernel): the lane only sets the A cursor.
__device__ __forceinline__ void mt_start_from(MtLane& g, uint32_t seed, uint32_t x397) {
  g.seed = seed;
  g.j = 0;
  g.a0 = seed;
  g.a1 = mt_seed_step(seed, 1);
  g.b = x397;
}

#ifndef YK_WALK_MAD
#define YK_WALK_MAD 1
#endif
// One seeding step whose index is wave-uniform (the walk's loop counter, in SGPRs): the multiply
// and the add of i as ONE v_mad_u64_u32 (low word of t * 1812433253 + i), three instructions
// instead of four (xor-shift, v_mul_lo_u32, v_add).  cmul holds 1812433253 in a VGPR: the
// instruction may read one SGPR operand, the 64-bit addend.
__device__ __forceinline__ uint32_t mt_seed_step_mad(uint32_t prev, uint64_t i, uint32_t cmul) {
  const uint32_t t = prev ^ (prev >> 30);
  uint64_t r, carry;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(r), "=s"(carry) : "v"(t), "v"(cmul), "s"(i));
  return (uint32_t)r;
}

// x_397 of the seeding sequence (random.hpp:69-81) for N seeds at once (independent chains
// interleaved for ILP).
template <int N>
__device__ __forceinline__ void mt_walk397xn(uint32_t (&x)[N]) {
#pragma unroll
  for (int k = 0; k < N; ++k) x[k] = mt_seed_step(x[k], 1);
#if YK_WALK_MAD
  uint32_t cmul;
  asm("v_mov_b32 %0, 0x6c078965" : "=v"(cmul));  // 1812433253
#pragma unroll 4
  for (uint32_t i = 2; i <= kMtM; ++i) {
#pragma unroll
    for (int k = 0; k < N; ++k) x[k] = mt_seed_step_mad(x[k], (uint64_t)i, cmul);
  }
#else
#pragma unroll 4
  for (uint32_t i = 2; i <= kMtM; ++i) {
#pragma unroll
    for (int k = 0; k < N; ++k) x[k] = mt_seed_step(x[k], i);
  }
#endif
}

// The rare path: the real engine in global scratch (seed :69-81, M_gen_rand :114-131).
// Out of line and by value so the hot path keeps the lane's cursors in registers.  At its first
// call (j = 227) cursor A holds x_227, and the seed x_0 is recovered from it: a seeding step
// x_i = C (u ^ u >> 30) + i is invertible (C odd: t = (x_i - i) C^-1 = u ^ u >> 30, and u = t ^
// t >> 30, since the xor changes only bits 0-1), so the lane never carries its seed.
constexpr uint32_t kMtSeedMulInv = 0x9638806du;  // 1812433253^-1 mod 2^32
__device__ __forceinline__ uint32_t mt_seed_from(uint32_t x, uint32_t i) {  // x_i -> x_0
  for (; i > 0; --i) {
    const uint32_t t = (x - i) * kMtSeedMulInv;
    x = t ^ (t >> 30);
  }
  return x;
}
__device__ __noinline__ uint32_t mt_slow(uint32_t* st, uint32_t x227, uint32_t j) {
  const uint32_t idx = j % kMtN;
  if (j == kLazyDraws) {
    uint32_t x = mt_seed_from(x227, kLazyDraws);
    st[0] = x;
    for (uint32_t i = 1; i < kMtN; ++i) {
      x = mt_seed_step(x, i);
      st[i] = x;
    }
  }
  if (j == kLazyDraws || idx == 0) {
    uint32_t k = 0;
    for (; k < kMtN - kMtM; ++k) st[k] = st[k + kMtM] ^ mt_mix(st[k], st[k + 1]);
    for (; k < kMtN - 1; ++k) st[k] = st[k + kMtM - kMtN] ^ mt_mix(st[k], st[k + 1]);
    st[kMtN - 1] = st[kMtM - 1] ^ mt_mix(st[kMtN - 1], st[0]);
  }
  return st[idx];
}

// The lazy cursors' draw without the check for the scratch engine: only for callers that know
// every lane drawing here has j + words <= kLazyDraws (rng_lazy_ok)
__device__ __forceinline__ uint32_t mt_next_lazy(MtLane& g) {
  const uint32_t z = g.b ^ mt_mix(g.a0, g.a1);
  g.a0 = g.a1;
  g.a1 = mt_seed_step(g.a1, g.j + 2);
  g.b = mt_seed_step(g.b, g.j + kMtM + 1);
  ++g.j;
  return mt_temper(z);
}
__device__ __forceinline__ bool rng_lazy_ok(const MtLane& g, uint32_t words) { return g.j + words <= kLazyDraws; }

__device__ __forceinline__ uint32_t mt_next(MtLane& g) {
  uint32_t z;
  if (g.j < kLazyDraws) {
    z = g.b ^ mt_mix(g.a0, g.a1);
    g.a0 = g.a1;
    g.a1 = mt_seed_step(g.a1, g.j + 2);
    g.b = mt_seed_step(g.b, g.j + kMtM + 1);
  } else {
    z = mt_slow(g.state, g.a0, g.j);  // (a0 = x_227 at the first call)
  }
  ++g.j;
  return mt_temper(z);
}

// Per-sample seed (include/ykgpu.h YK_SEED_*).  COUNTER: seed0 + (y*W + x)*spp + s in uint32
// arithmetic (source.cpp:154-158).  RANDOM_DEVICE: the call's 64-bit key hashed with the
// sample's 64-bit linear index (splitmix64 finaliser, high word) — one independent seed per
// sample, like the runtime build's std::random_device (source.cpp:159).
__device__ __forceinline__ uint32_t sample_seed(uint32_t mode, uint64_t key, uint32_t seed0, uint32_t y,
                                                uint32_t x, uint32_t W, uint32_t spp, uint32_t s) {
#ifndef YK_SEED_COUNTER_ONLY  // (A/B timing builds: the random-device mode compiled out)
  if (mode == 1u) {
    uint64_t z = key + (((uint64_t)y * W + x) * spp + s + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (uint32_t)(z >> 32);
  }
#endif
  return seed0 + (y * W + x) * spp + s;
}

// yk::xor128 (random.hpp:18-41): Marsaglia's xorshift128, the reference's other engine
// (YK_RNG_XOR128).  x, y, z start at their default member values and w = 88675123 ^ seed
// (:19-32); four words of state, so a sample needs neither the x_397 warm-up nor scratch.
struct X128Lane {
  uint32_t x, y, z, w;
  uint32_t n;  // words drawn (work counters only: dead in the production instances)
};
__device__ __forceinline__ void x128_start(X128Lane& g, uint32_t seed) {
  g.x = 123456789u;
  g.y = 362436069u;
  g.z = 521288629u;
  g.w = 88675123u ^ seed;
  g.n = 0;
}
__device__ __forceinline__ uint32_t x128_next(X128Lane& g) {  // operator(), :34-40
  const uint32_t t = g.x ^ (g.x << 11);
  g.x = g.y;
  g.y = g.z;
  g.z = g.w;
  g.w = (g.w ^ (g.w >> 19)) ^ (t ^ (t >> 8));
  ++g.n;
  return g.w;
}
__device__ __forceinline__ bool mt_used_fallback(const X128Lane&) { return false; }
__device__ __forceinline__ uint32_t rng_words(const X128Lane& g) { return g.n; }
__device__ __forceinline__ uint32_t rng_twists(const X128Lane&) { return 0u; }

__device__ __forceinline__ bool rng_lazy_ok(const X128Lane&, uint32_t) { return true; }

// One 32-bit draw of the lane's engine (kLazy: the caller has checked rng_lazy_ok)
template <bool kLazy = false>
__device__ __forceinline__ uint32_t rng_next(MtLane& g) { return kLazy ? mt_next_lazy(g) : mt_next(g); }
template <bool kLazy = false>
__device__ __forceinline__ uint32_t rng_next(X128Lane& g) { return x128_next(g); }

// generate_canonical<double,53> (random.hpp:161-183): two draws (both engines have
// min 0, max 2^32-1, so r = 2^32 and m = 2), sum = u0 + u1*2^32 rounded once, divided by 2^64
// (exact), clamped to 1 - eps/2.
template <bool kLazy = false, class G>
__device__ __forceinline__ double canonical(G& g) {
  const double u0 = (double)rng_next<kLazy>(g);
  const double u1 = (double)rng_next<kLazy>(g);
  // RN(u0 + u1 2^32) / 2^64 as ONE fma of the exactly scaled terms, u1 2^-32 + u0 2^-64: both
  // products are exact and a power-of-two scaling commutes with rounding in the normal range
  // (every term is 0 or >= 2^-64), so the result is the reference's bit for bit
  double r = __builtin_fma(u1, 0x1p-32, u0 * 0x1p-64);
  if (r >= 1.0) r = 1.0 - 0x1p-53;
  return r;
}
// uniform_real_distribution::operator() (random.hpp:273-278): c*(b-a)+a
template <bool kLazy = false, class G>
__device__ __forceinline__ double uniform(G& g, double a, double b) {
  return (canonical<kLazy>(g) * (b - a)) + a;
}
// uniform_real_distribution::operator() on an already drawn canonical c: the same c*(b-a)+a
// (Every call passes constant bounds.  (-1, 1): c*2 is exact, so c*2 + -1 is one fma with the same
// rounding; (0, 1): c*1 + 0 is c, as c >= 0.)
__device__ __forceinline__ double uniform_of(double c, double a, double b) {
  if (a == -1.0 && b == 1.0) return __builtin_fma(c, 2.0, -1.0);
  if (a == 0.0 && b == 1.0) return c;
  return (c * (b - a)) + a;
}
// Whether the next two words may be drawn speculatively and then given back by restoring a copy
// of the lane's engine: for mt19937 only inside the lazy cursors (the scratch engine's twist
// rewrites its state in place); xor128's state is the copy.
__device__ __forceinline__ bool rng_can_speculate(const MtLane& g) { return g.j + 2 <= kLazyDraws; }
__device__ __forceinline__ bool rng_can_speculate(const X128Lane&) { return true; }
// vec3::random(gen, -1, 1) (vec3.hpp:134-142): x, then y, then z
template <class G>
__device__ __forceinline__ v3 random_vec(G& g, double lo, double hi) {
  v3 r;
  r.x = uniform(g, lo, hi);
  r.y = uniform(g, lo, hi);
  r.z = uniform(g, lo, hi);
  return r;
}

// Schlick reflectance (dielectric extension; no reference code)
__device__ __forceinline__ double reflectance(double cosine, double ref_idx) {
  double r0 = (1 - ref_idx) / (1 + ref_idx);
  r0 = r0 * r0;
  const double x = 1 - cosine;
  return r0 + (1 - r0) * ((((x * x) * x) * x) * x);
}
// the same from r0 = ((1 - ref_idx) / (1 + ref_idx))^2 computed ahead (per material and side)
__device__ __forceinline__ double reflectance_r0(double cosine, double r0) {
  const double x = 1 - cosine;
  return r0 + (1 - r0) * ((((x * x) * x) * x) * x);
}

}  // namespace ykd
