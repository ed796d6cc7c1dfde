// yk_device_f32.hpp — per-lane arithmetic of one sample of render<float> (YK_PRECISION_FP32),
// gfx950 device code.
//
// yk::render<T> with T = float (source.cpp:98-99): geometry, camera, canonicals and math::sqrt
// in float; colours stay double (raytracer<T, double>, lambertian<double>), so the attenuation
// products and the per-pixel sum are the FP64 path's.  Every expression keeps the reference's
// C++ type promotions (a float meeting a double literal is promoted, e.g. near_zero's 1e-8 and
// the sky's `y + 1.0`) and its association order; the file is compiled with -ffp-contract=off,
// and float `/` and sqrtf are correctly rounded (hipcc's default
// -fhip-fp32-correctly-rounded-divide-sqrt; the parity tests check the results bit for bit
// against oracle/yk_oracle_path.h, which is pinned to the reference's own render<float>).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "yk_device.hpp"

namespace ykf {

struct v3 {
  float x, y, z;
};
__device__ __forceinline__ v3 add(v3 a, v3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ v3 sub(v3 a, v3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ v3 mul(v3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
__device__ __forceinline__ v3 divs(v3 a, float s) { return {a.x / s, a.y / s, a.z / s}; }
__device__ __forceinline__ v3 neg(v3 a) { return {-a.x, -a.y, -a.z}; }
__device__ __forceinline__ float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }  // vec3.hpp:145-147
__device__ __forceinline__ float len2(v3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }      // vec3.hpp:129
__device__ __forceinline__ v3 of(const double* p) { return {(float)p[0], (float)p[1], (float)p[2]}; }
__device__ __forceinline__ v3 off(const float* p) { return {p[0], p[1], p[2]}; }

// ---- float division without the special-case steps (the FP64 divs_fast's argument, yk_device.hpp)
// The compiler's correctly rounded float division on gfx950 is
//   div_scale(d), div_scale(n), rcp, fma, fma (refined reciprocal), mul, fma, fma, fma (two
//   residual corrections), div_fmas, div_fixup                        (11 instructions)
// div_scale rescales only when an exponent is extreme (|n / d| >= 2^96, d or 1/d or n / d
// denormal, |n| < 2^-104), div_fmas is then a plain fma, and div_fixup only rewrites NaN, inf,
// zero and denormal cases: for |n|, |d| in [2^-40, 2^40] (or n == 0) the sequence below is the same
// arithmetic minus those three steps, and the refined reciprocal, which depends only on d, serves
// every component of a vector.  A zero numerator's sign is fixed as in ykd::div_by.  Checked bit
// for bit against IEEE float division on the GPU (ykgpu_math_div_f32,
// tests/test_gpu_parity.py::test_fast_float_division_is_ieee_division).
__device__ __forceinline__ bool div_range(float x) { return fabsf(x) >= 0x1p-40f && fabsf(x) <= 0x1p40f; }
__device__ __forceinline__ bool num_range(float x) { return x == 0.0f || div_range(x); }
__device__ __forceinline__ float rcp_refined(float d) {
  const float r0 = __builtin_amdgcn_rcpf(d);
  return __builtin_fmaf(__builtin_fmaf(-d, r0, 1.0f), r0, r0);
}
__device__ __forceinline__ float div_by(float n, float d, float r) {
  const float q0 = n * r;
  const float q1 = __builtin_fmaf(__builtin_fmaf(-d, q0, n), r, q0);
  return __builtin_copysignf(__builtin_fmaf(__builtin_fmaf(-d, q1, n), r, q1), q0);
}
// vector / scalar with the shared reciprocal r = rcp_refined(d); a wave with any operand out of
// range recomputes with the full division (same bits for the in-range lanes)
__device__ __forceinline__ v3 divs_fast_r(v3 a, float d, float r) {
  v3 q = {div_by(a.x, d, r), div_by(a.y, d, r), div_by(a.z, d, r)};
  const bool ok = div_range(d) && num_range(a.x) && num_range(a.y) && num_range(a.z);
  if (__builtin_expect(__ballot(!ok) != 0, 0)) q = divs(a, d);
  return q;
}
__device__ __forceinline__ v3 divs_fast(v3 a, float d) { return divs_fast_r(a, d, rcp_refined(d)); }

// math::sqrt<float> (math.hpp:10-19): `T x = s / 2.0` and `x = (x + s / x) / 2.0` halve in
// double and round to float, which equals the float product by 0.5f (halving is exact, so both
// are one rounding of the same value).  As for FP64 (yk_device.hpp), the loop's result is a
// fixed point that does not depend on the start: for every positive float s in [2^-100, 2^100]
// the loop started at the correctly rounded sqrtf(s) ends at the reference's value (checked
// exhaustively over all 2^31 positive floats by tools/fsqrt_check.c: every float terminates,
// at most 80 reference iterations, and only one input — outside that range — differs).  One
// step from sqrtf(s) already lands on that fixed point (the argument of DESIGN.md §3 holds for any
// binary format; tools/fsqrt_check.c confirms it for every float in [2^-100, 2^100]), so inside
// the range the device returns it without the confirming second division.
__device__ __forceinline__ float nsqrt(float s, uint32_t& iters) {
  if (s >= 0x1p-100f && s <= 0x1p100f) {
    const float r = __builtin_sqrtf(s);
    ++iters;
    // s / r without div_scale / div_fmas / div_fixup: for s in [2^-100, 2^100], r, 1/r and s / r
    // lie in [2^-50, 2^50], where none of them changes anything (see div_by)
    return (r + div_by(s, r, rcp_refined(r))) * 0.5f;
  }
  float x = s * 0.5f;
  float prev = 0.0f;
  for (int guard = 0; x != prev && guard < 4096; ++guard) {  // the bound only matters for NaN/inf
    prev = x;
    x = (x + s / x) * 0.5f;
    ++iters;
  }
  return x;
}

// reflect(): vec3.hpp:199-202, v - (2*dot(v,n))*n with `2 * dot` a float product
__device__ __forceinline__ v3 reflect(v3 v, v3 n) { return sub(v, mul(n, 2.0f * dot(v, n))); }
// near_zero(): vec3.hpp:76-80 — s = 1e-8 is a double, so |x| is compared after promotion; the
// reference tests x twice and never z
__device__ __forceinline__ bool near_zero(v3 a) {
  const float ax = a.x > 0 ? a.x : -a.x, ay = a.y > 0 ? a.y : -a.y;
  return ((double)ax < 1e-8) && ((double)ay < 1e-8) && ((double)ax < 1e-8);
}

// generate_canonical<float, 24> (random.hpp:161-183): m = max(1, (24 + 32) / 33) = 1 draw;
// sum = float(u) (rounded to nearest), ret = sum / 2^32 (exact scaling), clamped to 1 - eps/2.
// (kLazy: the caller has checked ykd::rng_lazy_ok for the words it draws)
template <bool kLazy = false, class G>
__device__ __forceinline__ float canonical(G& g) {
  const float sum = (float)ykd::rng_next<kLazy>(g);
  float r = sum * 0x1p-32f;
  if (r >= 1.0f) r = 1.0f - 0x1p-24f;
  return r;
}
// uniform_real_distribution<float>::operator() (random.hpp:273-278): c*(b-a)+a in float
__device__ __forceinline__ float uniform_of(float c, float a, float b) { return (c * (b - a)) + a; }
template <class G>
__device__ __forceinline__ float uniform(G& g, float a, float b) { return uniform_of(ykf::canonical(g), a, b); }
// vec3<float>::random(gen, -1, 1) (vec3.hpp:134-142): x, then y, then z
template <class G>
__device__ __forceinline__ v3 random_vec(G& g, float lo, float hi) {
  v3 r;
  r.x = ykf::uniform(g, lo, hi);
  r.y = ykf::uniform(g, lo, hi);
  r.z = ykf::uniform(g, lo, hi);
  return r;
}

// Schlick reflectance (dielectric extension; no reference code), in float
__device__ __forceinline__ float reflectance(float cosine, float ref_idx) {
  float r0 = (1.0f - ref_idx) / (1.0f + ref_idx);
  r0 = r0 * r0;
  const float x = 1.0f - cosine;
  return r0 + (1.0f - r0) * ((((x * x) * x) * x) * x);
}

}  // namespace ykf
