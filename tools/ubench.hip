// tools/ubench.hip — issue cost of single VALU instructions / short sequences on gfx950: one
// wave per SIMD, eight independent chains, clock64() around the loop.  Diagnostic only: says
// which FP64 / integer operations the render loop should avoid.
//   build: hipcc -O3 --offload-arch=gfx950 -o tools/ubench tools/ubench.hip ; run: tools/ubench [out.jsonl]
// The JSON lines are the evidence of the roofline's FP64 VALU peak (profiles/r03_ubench.jsonl,
// tools/valu_peak.py, bench.py).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cmath>
#include <cstdio>

constexpr int kChains = 8;
constexpr int kIters = 2048;

struct FmaF32 {
  using T = float;
  static __device__ void op(T& x, T a, T b) { asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x) : "v"(a), "v"(b)); }
};
struct PkFmaF32 {
  using T = double;  // two packed floats in a 64-bit register pair
  static __device__ void op(T& x, T a, T b) { asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(x) : "v"(a), "v"(b)); }
};
struct FmaMixF32 {  // the BVH slab FMA with a binary16 plane (yk_bvh.hpp HalfNode)
  using T = float;
  static __device__ void op(T& x, T a, T b) {
    asm volatile("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,0,0]" : "+v"(x) : "v"(a), "v"(b));
  }
};
struct FmaF64 {
  using T = double;
  static __device__ void op(T& x, T a, T b) { asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(x) : "v"(a), "v"(b)); }
};
struct MulF64 {
  using T = double;
  static __device__ void op(T& x, T a, T) { asm volatile("v_mul_f64 %0, %1, %0" : "+v"(x) : "v"(a)); }
};
struct AddF64 {
  using T = double;
  static __device__ void op(T& x, T a, T) { asm volatile("v_add_f64 %0, %1, %0" : "+v"(x) : "v"(a)); }
};
struct RcpF64 {
  using T = double;
  static __device__ void op(T& x, T, T) { asm volatile("v_rcp_f64 %0, %0" : "+v"(x)); }
};
struct RsqF64 {
  using T = double;
  static __device__ void op(T& x, T, T) { asm volatile("v_rsq_f64 %0, %0" : "+v"(x)); }
};
struct SqrtF64 {
  using T = double;
  static __device__ void op(T& x, T, T) { asm volatile("v_sqrt_f64 %0, %0" : "+v"(x)); }
};
struct RcpF32 {
  using T = float;
  static __device__ void op(T& x, T, T) { asm volatile("v_rcp_f32 %0, %0" : "+v"(x)); }
};
struct MinMax3F32 {
  using T = float;
  static __device__ void op(T& x, T a, T b) { asm volatile("v_max3_f32 %0, %1, %2, %0" : "+v"(x) : "v"(a), "v"(b)); }
};
struct CmpF64 {  // compare + select, the shape of the culling tests (compiler generated)
  using T = double;
  static __device__ void op(T& x, T a, T b) { x = (x < a) ? b : x + b; asm volatile("" : "+v"(x)); }
};
struct MulLoU32 {
  using T = uint32_t;
  static __device__ void op(T& x, T a, T) { asm volatile("v_mul_lo_u32 %0, %1, %0" : "+v"(x) : "v"(a)); }
};
struct MadU64U32 {  // the walk step's multiply-add (low word of t * c + i), addend from SGPRs
  using T = uint32_t;
  static __device__ void op(T& x, T a, T) {
    uint64_t r, cc;
    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 7" : "=v"(r), "=s"(cc) : "v"(x), "v"(a));
    x = (uint32_t)r;
  }
};
struct XorShrU32 {  // x ^ (x >> 30): the seeding step's shift-xor
  using T = uint32_t;
  static __device__ void op(T& x, T, T) {
    uint32_t t;
    asm volatile("v_lshrrev_b32 %1, 30, %0\n\tv_xor_b32 %0, %0, %1" : "+v"(x), "=&v"(t));
  }
};
// round 5 (the lane-op roofline's per-class issue costs, uecraytracing_amd/flops.py): one plain
// 32-bit op, gfx950's three-input bitwise op, the u32 -> f64 conversion of every engine word, and
// the seed walk's whole step as the kernel issues it (v_lshrrev + v_xor + v_mad_u64_u32)
struct XorB32 {
  using T = uint32_t;
  static __device__ void op(T& x, T a, T) { asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x) : "v"(a)); }
};
struct Bitop3B32 {
  using T = uint32_t;
  static __device__ void op(T& x, T a, T b) { asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x78" : "+v"(x) : "v"(a), "v"(b)); }
};
struct CvtF64U32 {
  using T = double;
  static __device__ void op(T& x, T, T) { asm volatile("v_cvt_f64_u32 %0, 7" : "=v"(x)); }
};
struct WalkStep {
  using T = uint32_t;
  static __device__ void op(T& x, T a, T) {
    uint32_t t;
    uint64_t r, cc;
    asm volatile("v_lshrrev_b32 %0, 30, %1\n\tv_xor_b32 %0, %1, %0" : "=&v"(t) : "v"(x));
    asm volatile("v_mad_u64_u32 %0, %1, %2, %3, 7" : "=v"(r), "=s"(cc) : "v"(t), "v"(a));
    x = (uint32_t)r;
  }
};
struct CmpLtF64 {  // v_cmp into an SGPR pair, then used by a cndmask so it is not dead
  using T = uint32_t;
  static __device__ void op(T& x, T a, T b) {
    const double da = (double)a, db = (double)b;
    asm volatile("v_cmp_lt_f64_e64 s[40:41], %1, %2\n\tv_cndmask_b32_e64 %0, %0, 1, s[40:41]" : "+v"(x) : "v"(da), "v"(db) : "s40", "s41");
  }
};
struct CmpClassF64 {
  using T = uint32_t;
  static __device__ void op(T& x, T a, T) {
    const double da = (double)a;
    const uint32_t m = 0x60u;
    asm volatile("v_cmp_class_f64_e64 s[40:41], %1, %2\n\tv_cndmask_b32_e64 %0, %0, 1, s[40:41]" : "+v"(x) : "v"(da), "v"(m) : "s40", "s41");
  }
};
struct CmpLtU32 {
  using T = uint32_t;
  static __device__ void op(T& x, T a, T) {
    asm volatile("v_cmp_lt_u32_e64 s[40:41], %0, %1\n\tv_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(x) : "v"(a) : "s40", "s41");
  }
};
struct CndOnly {
  using T = uint32_t;
  static __device__ void op(T& x, T a, T) {
    asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(x) : "v"(a) : "s40", "s41");
  }
};
struct DivScaleF64 {
  using T = double;
  static __device__ void op(T& x, T a, T) { asm volatile("v_div_scale_f64 %0, vcc, %0, %1, %0" : "+v"(x) : "v"(a) : "vcc"); }
};
struct DivFixupF64 {
  using T = double;
  static __device__ void op(T& x, T a, T b) { asm volatile("v_div_fixup_f64 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b)); }
};
struct DivFmasF64 {
  using T = double;
  static __device__ void op(T& x, T a, T b) { asm volatile("s_mov_b64 vcc, 0\n\tv_div_fmas_f64 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b) : "vcc"); }
};
struct BfeU32 {
  using T = uint32_t;
  static __device__ void op(T& x, T, T) { asm volatile("v_bfe_u32 %0, %0, 20, 11" : "+v"(x)); }
};
// whole sequences, compiler generated (not asm): correctly rounded division and sqrt
struct DivF64 {
  using T = double;
  static __device__ void op(T& x, T a, T) { x = a / x; asm volatile("" : "+v"(x)); }
};
struct SqrtLibF64 {
  using T = double;
  static __device__ void op(T& x, T, T) { x = __builtin_sqrt(x); asm volatile("" : "+v"(x)); }
};

template <class Op>
__global__ __launch_bounds__(64) void bench(uint64_t* cyc, uint64_t* rt, typename Op::T* sink, typename Op::T a,
                                            typename Op::T b, typename Op::T init) {
  using T = typename Op::T;
  T x[kChains];
#pragma unroll
  for (int k = 0; k < kChains; ++k) x[k] = init;
  const uint64_t r0 = wall_clock64();
  const uint64_t t0 = clock64();
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int k = 0; k < kChains; ++k) Op::op(x[k], a, b);
  }
  const uint64_t t1 = clock64();
  const uint64_t r1 = wall_clock64();
  T s = x[0];
#pragma unroll
  for (int k = 1; k < kChains; ++k) s = s + x[k];
  sink[blockIdx.x * 64 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0, rt[blockIdx.x] = r1 - r0;
}

// JSON lines of the run (one per op and occupancy) for profiles/: ticks = shader clock cycles
// (s_memtime); waves_per_simd = waves / (4 x CUs); simd_cycles_per_instr = ticks per op per wave
// / waves_per_simd (the SIMD's issue cost of one wave64 instruction once it is saturated);
// clock_mhz = ticks / s_memrealtime ticks x 100 MHz (the clock the chip held under this loop)
static FILE* g_json = nullptr;
static int g_cus = 0;

// Chip-level throughput of one op: every SIMD holds `wps` waves of the same stream, the whole
// launch timed with HIP events: lane-flops / elapsed.  The peak the roofline divides by is the
// best of these for v_fma_f64 (tools/valu_peak.py).
template <class Op>
__global__ __launch_bounds__(64) void chip(typename Op::T* sink, typename Op::T a, typename Op::T b,
                                           typename Op::T init, int iters) {
  using T = typename Op::T;
  T x[kChains];
#pragma unroll
  for (int k = 0; k < kChains; ++k) x[k] = init;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < kChains; ++k) Op::op(x[k], a, b);
  }
  T s = x[0];
#pragma unroll
  for (int k = 1; k < kChains; ++k) s = s + x[k];
  sink[blockIdx.x * 64 + threadIdx.x] = s;
}

template <class Op>
void chip_rate(const char* name, double flops_per_lane_op, typename Op::T a, typename Op::T b,
               typename Op::T init, int wps) {
  using T = typename Op::T;
  const int waves = wps * 4 * g_cus, iters = 16384;
  T* sink;
  (void)hipMalloc(&sink, (size_t)waves * 64 * sizeof(T));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 4; ++rep) {
    (void)hipEventRecord(e0, 0);
    hipLaunchKernelGGL(chip<Op>, dim3(waves), dim3(64), 0, 0, sink, a, b, init, iters);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep > 0 && ms < best) best = ms;  // the first launch warms the clock
  }
  const double ops = (double)waves * iters * kChains;  // wave-instructions
  const double tf = ops * 64 * flops_per_lane_op / (best * 1e-3) / 1e12;
  const double cyc = (best * 1e-3) * 2.4e9 * 4 * g_cus / ops;  // SIMD cycles per wave-instr at 2.4 GHz
  printf("chip %-12s waves/SIMD=%d  %.3f ms  %.2f TFLOP/s  (%.2f SIMD cycles per wave-instruction at 2.4 GHz)\n",
         name, wps, best, tf, cyc);
  if (g_json)
    fprintf(g_json,
            "{\"chip_op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"wave_instructions\": %.0f, "
            "\"flops_per_lane_op\": %.0f, \"tflops\": %.3f, \"simd_cycles_per_instr_at_2400mhz\": %.4f}\n",
            name, wps, best, ops, flops_per_lane_op, tf, cyc);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  (void)hipFree(sink);
}

template <class Op>
void run(const char* name, typename Op::T a, typename Op::T b, typename Op::T init, int waves) {
  using T = typename Op::T;
  uint64_t *cyc, *rt;
  T* sink;
  (void)hipMalloc(&cyc, waves * sizeof(uint64_t));
  (void)hipMalloc(&rt, waves * sizeof(uint64_t));
  (void)hipMalloc(&sink, waves * 64 * sizeof(T));
  hipLaunchKernelGGL(bench<Op>, dim3(waves), dim3(64), 0, 0, cyc, rt, sink, a, b, init);
  hipLaunchKernelGGL(bench<Op>, dim3(waves), dim3(64), 0, 0, cyc, rt, sink, a, b, init);
  (void)hipDeviceSynchronize();
  static uint64_t h[8192], hr[8192];
  (void)hipMemcpy(h, cyc, waves * sizeof(uint64_t), hipMemcpyDeviceToHost);
  (void)hipMemcpy(hr, rt, waves * sizeof(uint64_t), hipMemcpyDeviceToHost);
  double mean = 0, mrt = 0;
  for (int i = 0; i < waves; ++i) mean += (double)h[i], mrt += (double)hr[i];
  mean /= waves;
  mrt /= waves;
  const double per_wave = mean / ((double)kIters * kChains);
  const double wps = (double)waves / (4.0 * g_cus);
  printf("%-12s waves=%5d  %.2f clock64 ticks per op per wave  (%.2f SIMD cycles per wave-instruction, clock %.0f MHz)\n",
         name, waves, per_wave, per_wave / wps, mean / mrt * 100.0);
  if (g_json)
    fprintf(g_json,
            "{\"op\": \"%s\", \"waves\": %d, \"waves_per_simd\": %.3f, \"ticks_per_op_per_wave\": %.4f, "
            "\"simd_cycles_per_instr\": %.4f, \"clock_mhz\": %.1f}\n",
            name, waves, wps, per_wave, per_wave / wps, mean / mrt * 100.0);
  (void)hipFree(cyc);
  (void)hipFree(rt);
  (void)hipFree(sink);
}

// accuracy of the hardware approximations (max error in units of 2^-52 relative)
__global__ void approx(const double* in, double* out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double x = in[i], r, s, q;
  asm volatile("v_rsq_f64 %0, %1" : "=v"(r) : "v"(x));
  asm volatile("v_sqrt_f64 %0, %1" : "=v"(s) : "v"(x));
  asm volatile("v_rcp_f64 %0, %1" : "=v"(q) : "v"(x));
  out[3 * i] = r;
  out[3 * i + 1] = s;
  out[3 * i + 2] = q;
}

void accuracy() {
  const uint64_t n = 1 << 22;
  double* h = new double[n];
  double* o = new double[3 * n];
  uint64_t st = 88172645463325252ull;
  for (uint64_t i = 0; i < n; ++i) {
    st ^= st << 13, st ^= st >> 7, st ^= st << 17;
    const double m = 1.0 + (double)(st >> 11) * 0x1p-53;
    const int e = (int)((st >> 3) % 1200) - 600;
    h[i] = __builtin_ldexp(m, e);
  }
  double *d_in, *d_out;
  (void)hipMalloc(&d_in, n * 8);
  (void)hipMalloc(&d_out, 3 * n * 8);
  (void)hipMemcpy(d_in, h, n * 8, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(approx, dim3((n + 255) / 256), dim3(256), 0, 0, d_in, d_out, n);
  (void)hipMemcpy(o, d_out, 3 * n * 8, hipMemcpyDeviceToHost);
  long double worst[3] = {0, 0, 0};
  for (uint64_t i = 0; i < n; ++i) {
    const long double x = h[i], sq = sqrtl(x);
    const long double ref[3] = {1.0L / sq, sq, 1.0L / x};
    for (int k = 0; k < 3; ++k) {
      long double e = ((long double)o[3 * i + k] - ref[k]) / ref[k];
      if (e < 0) e = -e;
      if (e > worst[k]) worst[k] = e;
    }
  }
  printf("max relative error / 2^-52:  rsq %.3Lg   sqrt %.3Lg   rcp %.3Lg\n", worst[0] * 0x1p52L,
         worst[1] * 0x1p52L, worst[2] * 0x1p52L);
}

int main(int argc, char** argv) {
  // argv[1]: optional path of the JSON-lines summary
  if (argc > 1) g_json = fopen(argv[1], "w");
  accuracy();
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, 0);
  g_cus = p.multiProcessorCount;
  printf("%s  CUs %d  clock %d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  if (g_json) fprintf(g_json, "{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d}\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  for (int wps : {1, 2, 4, 8}) {
    chip_rate<FmaF32>("fma_f32", 2, 1.0000001f, 0.5f, 1.0f, wps);
    chip_rate<PkFmaF32>("pk_fma_f32", 4, 1.0, 0.5, 1.0, wps);
    chip_rate<FmaMixF32>("fma_mix_f32", 2, 1.0f, 0.5f, 1.0f, wps);
    chip_rate<FmaF64>("fma_f64", 2, 1.0000001, 0.5, 1.0, wps);
    chip_rate<MulLoU32>("mul_lo_u32", 0, 1812433253u, 0, 7u, wps);
    chip_rate<MadU64U32>("mad_u64_u32", 0, 1812433253u, 0, 7u, wps);
    chip_rate<XorShrU32>("xor_shr_u32", 0, 0, 0, 7u, wps);
    chip_rate<XorB32>("xor_b32", 0, 0x5bd1e995u, 0, 7u, wps);
    chip_rate<Bitop3B32>("bitop3_b32", 0, 0x5bd1e995u, 0x9908b0dfu, 7u, wps);
    chip_rate<CvtF64U32>("cvt_f64_u32", 0, 0, 0, 1.0, wps);
    chip_rate<WalkStep>("walk_step", 0, 1812433253u, 0, 7u, wps);
  }
  for (int waves : {p.multiProcessorCount * 4, p.multiProcessorCount * 8, p.multiProcessorCount * 16}) {
    run<FmaF32>("fma_f32", 1.0000001f, 0.5f, 1.0f, waves);
    run<PkFmaF32>("pk_fma_f32", 1.0, 0.5, 1.0, waves);
    run<MinMax3F32>("max3_f32", 1.0f, 0.5f, 1.0f, waves);
    run<RcpF32>("rcp_f32", 0, 0, 1.5f, waves);
    run<FmaF64>("fma_f64", 1.0000001, 0.5, 1.0, waves);
    run<MulF64>("mul_f64", 1.0000001, 0, 1.0, waves);
    run<AddF64>("add_f64", 1e-9, 0, 1.0, waves);
    run<CmpF64>("cmp+add_f64", 2.0, 1e-9, 1.0, waves);
    run<RcpF64>("rcp_f64", 0, 0, 1.5, waves);
    run<RsqF64>("rsq_f64", 0, 0, 1.5, waves);
    run<SqrtF64>("v_sqrt_f64", 0, 0, 1.5, waves);
    run<DivF64>("div_f64 seq", 1.5, 0, 1.2, waves);
    run<SqrtLibF64>("sqrt_f64 seq", 0, 0, 1.5, waves);
    run<MulLoU32>("mul_lo_u32", 1812433253u, 0, 7u, waves);
    run<CmpLtF64>("cmp_f64+cnd", 2u, 3u, 1u, waves);
    run<CmpClassF64>("cls_f64+cnd", 2u, 0, 1u, waves);
    run<CmpLtU32>("cmp_u32+cnd", 5u, 0, 7u, waves);
    run<CndOnly>("cndmask", 5u, 0, 7u, waves);
    run<DivScaleF64>("div_scale", 1.5, 0, 1.25, waves);
    run<DivFixupF64>("div_fixup", 1.5, 1.25, 1.2, waves);
    run<DivFmasF64>("div_fmas", 1.0000001, 1e-9, 1.0, waves);
    run<BfeU32>("bfe_u32", 0, 0, 0x3ff00000u, waves);
    run<XorShrU32>("xor_shr_u32", 0, 0, 7u, waves);
  }
  if (g_json) fclose(g_json);
  return 0;
}
