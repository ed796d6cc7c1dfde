// tools/flopcal.hip — calibrates the FP64/FP32 VALU flop counters of rocprofv3 on gfx950 against
// known instruction counts, so the render kernel's SQ_INSTS_VALU_FLOPS_FP64 can be read as flops
// (VERDICT r01 "What's weak" 3).  One dispatch per case, each a known number of FP64 / FP32
// instructions per active lane, with all 64 lanes or only some of them active:
//   case  op              active lanes per wave   per-lane flops (FMA = 2)
// Expected per dispatch = waves * active * kIters * kChains * flops_per_op.
//   build: hipcc -O3 --offload-arch=gfx950 -o tools/flopcal tools/flopcal.hip
//   run:   rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP32
//            SQ_INSTS_VALU -d <dir> -o run -- tools/flopcal
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int kChains = 8;
constexpr int kIters = 1024;
constexpr int kBlocks = 1024;  // 4 waves each

struct FmaF64 {
  using T = double;
  static constexpr int kFlops = 2;
  static __device__ void op(T& x, T a, T b) { asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(x) : "v"(a), "v"(b)); }
};
struct MulF64 {
  using T = double;
  static constexpr int kFlops = 1;
  static __device__ void op(T& x, T a, T) { asm volatile("v_mul_f64 %0, %1, %0" : "+v"(x) : "v"(a)); }
};
struct AddF64 {
  using T = double;
  static constexpr int kFlops = 1;
  static __device__ void op(T& x, T a, T) { asm volatile("v_add_f64 %0, %1, %0" : "+v"(x) : "v"(a)); }
};
struct RcpF64 {
  using T = double;
  static constexpr int kFlops = 1;
  static __device__ void op(T& x, T, T) { asm volatile("v_rcp_f64 %0, %0" : "+v"(x)); }
};
struct FmaF32 {
  using T = float;
  static constexpr int kFlops = 2;
  static __device__ void op(T& x, T a, T b) { asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(x) : "v"(a), "v"(b)); }
};
struct PkFmaF32 {
  using T = double;  // two packed floats
  static constexpr int kFlops = 4;
  static __device__ void op(T& x, T a, T b) { asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(x) : "v"(a), "v"(b)); }
};

// the other FP64 instructions the render kernel issues: do the FLOPS/ADD/MUL/FMA/TRANS counters see them?
struct DivScaleF64 {
  using T = double;
  static constexpr int kFlops = 0;
  static __device__ void op(T& x, T a, T) { asm volatile("v_div_scale_f64 %0, vcc, %0, %1, %0" : "+v"(x) : "v"(a) : "vcc"); }
};
struct DivFmasF64 {
  using T = double;
  static constexpr int kFlops = 2;
  static __device__ void op(T& x, T a, T b) { asm volatile("s_mov_b64 vcc, 0\n\tv_div_fmas_f64 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b) : "vcc"); }
};
struct DivFixupF64 {
  using T = double;
  static constexpr int kFlops = 0;
  static __device__ void op(T& x, T a, T b) { asm volatile("v_div_fixup_f64 %0, %0, %1, %2" : "+v"(x) : "v"(a), "v"(b)); }
};
struct MaxF64 {
  using T = double;
  static constexpr int kFlops = 0;
  static __device__ void op(T& x, T a, T) { asm volatile("v_max_f64 %0, %1, %0" : "+v"(x) : "v"(a)); }
};
struct CvtF64U32 {
  using T = double;
  static constexpr int kFlops = 0;
  static __device__ void op(T& x, T a, T) { asm volatile("v_cvt_f64_u32 %0, %1" : "=v"(x) : "v"((uint32_t)a)); }
};
struct CvtF32F64 {
  using T = double;
  static constexpr int kFlops = 0;
  static __device__ void op(T& x, T, T) {
    float f;
    asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f) : "v"(x));
    x = (double)f;
  }
};
struct CmpF64 {
  using T = double;
  static constexpr int kFlops = 0;
  static __device__ void op(T& x, T a, T) { asm volatile("v_cmp_lt_f64 vcc, %0, %1" : "+v"(x) : "v"(a) : "vcc"); }
};
struct LdexpF64 {
  using T = double;
  static constexpr int kFlops = 0;
  static __device__ void op(T& x, T, T) { asm volatile("v_ldexp_f64 %0, %0, 1" : "+v"(x)); }
};

template <class Op>
__global__ __launch_bounds__(256) void cal(typename Op::T* sink, typename Op::T a, typename Op::T b,
                                           typename Op::T init, uint32_t active) {
  using T = typename Op::T;
  T x[kChains];
#pragma unroll
  for (int k = 0; k < kChains; ++k) x[k] = init;
  if ((threadIdx.x & 63u) < active) {
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
      for (int k = 0; k < kChains; ++k) Op::op(x[k], a, b);
    }
  }
  T s = x[0];
#pragma unroll
  for (int k = 1; k < kChains; ++k) s = s + x[k];
  sink[blockIdx.x * 256 + threadIdx.x] = s;
}

template <class Op>
void run(const char* name, uint32_t active, typename Op::T a, typename Op::T b, typename Op::T init) {
  using T = typename Op::T;
  T* sink;
  (void)hipMalloc(&sink, (size_t)kBlocks * 256 * sizeof(T));
  hipLaunchKernelGGL(cal<Op>, dim3(kBlocks), dim3(256), 0, 0, sink, a, b, init, active);
  (void)hipDeviceSynchronize();
  (void)hipFree(sink);
  const double waves = kBlocks * 4.0;
  printf("case %-10s active %2u  wave-instr %.6g  lane-flops %.6g\n", name, active,
         waves * kIters * kChains, waves * active * kIters * kChains * (double)Op::kFlops);
}

int main() {
  // dispatch order = the order of the rows printed (rocprofv3 Dispatch_Id)
  for (uint32_t act : {64u, 16u}) {
    run<FmaF64>("fma_f64", act, 1.0000001, 0.5, 1.0);
    run<MulF64>("mul_f64", act, 1.0000001, 0, 1.0);
    run<AddF64>("add_f64", act, 1e-9, 0, 1.0);
    run<RcpF64>("rcp_f64", act, 0, 0, 1.5);
    run<FmaF32>("fma_f32", act, 1.0000001f, 0.5f, 1.0f);
    run<PkFmaF32>("pk_fma_f32", act, 1.0, 0.5, 1.0);
  }
  run<DivScaleF64>("div_scale", 64, 1.5, 0, 1.25);
  run<DivFmasF64>("div_fmas", 64, 1.0000001, 1e-9, 1.0);
  run<DivFixupF64>("div_fixup", 64, 1.5, 1.25, 1.2);
  run<MaxF64>("max_f64", 64, 1.5, 0, 1.2);
  run<CvtF64U32>("cvt_f64_u32", 64, 7.0, 0, 1.0);
  run<CvtF32F64>("cvt_f32_f64", 64, 0, 0, 1.0);  // + one v_cvt_f64_f32 per op
  run<CmpF64>("cmp_f64", 64, 1.5, 0, 1.2);
  run<LdexpF64>("ldexp_f64", 64, 0, 0, 1.0);
  return 0;
}
