// tools/walkbench.hip — throughput of the mt19937 seeding step x' = 1812433253 (x ^ (x >> 30)) + i
// (random.hpp:69-81) in several instruction forms, over a full-GPU grid with 4 interleaved chains
// per thread (the warm-up kernel's shape).  Diagnostic only: picks the form yk_device.hpp uses.
//   build: hipcc -O3 --offload-arch=gfx950 -o /tmp/walkbench tools/walkbench.hip ; run: /tmp/walkbench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

constexpr uint32_t kC = 1812433253u;  // 0x6C078965 = 0x6C * 2^24 + 0x078965 = 0x6C07 * 2^16 + 0x8965

__device__ __forceinline__ uint32_t xs(uint32_t x) { return x ^ (x >> 30); }

// the compiler's form of the C expression (v_mul_lo_u32 + v_add)
struct Plain {
  static __device__ __forceinline__ uint32_t step(uint32_t x, uint32_t i) { return kC * xs(x) + i; }
};
// one v_mad_u64_u32 for the multiply-add (low half)
struct Mad64 {
  static __device__ __forceinline__ uint32_t step(uint32_t x, uint32_t i) {
    const uint32_t t = xs(x);
    uint64_t r;
    asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(r) : "v"(t), "s"(kC), "v"((uint64_t)i) : "vcc");
    return (uint32_t)r;
  }
};
// 24-bit pieces: v_mul/mad_u32_u24 read the low 24 bits of their operands, so
// t C = t24 * 0x078965 + ((t >> 24) * 0x078965 + t24 * 0x6C) << 24   (mod 2^32)
struct U24 {
  static __device__ __forceinline__ uint32_t step(uint32_t x, uint32_t i) {
    const uint32_t t = xs(x);
    uint32_t a, c, b, r;
    asm volatile(
        "v_mad_u32_u24 %0, %4, %5, %6\n\t"
        "v_mul_u32_u24 %1, %4, %7\n\t"
        "v_lshrrev_b32 %2, 24, %4\n\t"
        "v_mad_u32_u24 %1, %2, %5, %1\n\t"
        "v_lshl_add_u32 %3, %1, 24, %0"
        : "=&v"(a), "=&v"(c), "=&v"(b), "=v"(r)
        : "v"(t), "s"(0x078965u), "v"(i), "s"(0x6Cu));
    return r;
  }
};
// 16-bit pieces with op_sel (no extraction): t C = tl * 0x8965 + ((th * 0x8965 + tl * 0x6C07) << 16)
struct U16 {
  static __device__ __forceinline__ uint32_t step(uint32_t x, uint32_t i) {
    const uint32_t t = xs(x);
    uint32_t a, m, r;
    asm volatile(
        "v_mad_u32_u16 %0, %3, %4, %5\n\t"
        "v_mad_u32_u16 %1, %3, %4, 0 op_sel:[1,0,0,0]\n\t"
        "v_mad_u32_u16 %1, %3, %6, %1\n\t"
        "v_lshl_add_u32 %2, %1, 16, %0"
        : "=&v"(a), "=&v"(m), "=v"(r)
        : "v"(t), "s"(0x8965u), "v"(i), "s"(0x6C07u));
    return r;
  }
};

template <class S>
__global__ __launch_bounds__(256) void walk(uint32_t* out, uint32_t reps) {
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t x[4] = {gid * 4 + 1, gid * 4 + 2, gid * 4 + 3, gid * 4 + 4};
  for (uint32_t r = 0; r < reps; ++r) {
#pragma unroll 4
    for (uint32_t i = 1; i <= 397; ++i) {
#pragma unroll
      for (int k = 0; k < 4; ++k) x[k] = S::step(x[k], i);
    }
  }
  out[gid] = x[0] ^ x[1] ^ x[2] ^ x[3];
}

template <class S>
double run(const char* name, uint32_t* d, int blocks, uint32_t reps, std::vector<uint32_t>& res) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  hipLaunchKernelGGL(walk<S>, dim3(blocks), dim3(256), 0, 0, d, 1u);
  (void)hipEventRecord(a);
  hipLaunchKernelGGL(walk<S>, dim3(blocks), dim3(256), 0, 0, d, reps);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  res.resize((size_t)blocks * 256);
  (void)hipMemcpy(res.data(), d, res.size() * 4, hipMemcpyDeviceToHost);
  const double steps = (double)blocks * 256 * 4 * 397 * reps;
  printf("%-6s %8.3f ms  %.3f Gsteps/s\n", name, ms, steps / ms / 1e6);
  return ms;
}

int main() {
  const int blocks = 256 * 32;
  const uint32_t reps = 16;
  uint32_t* d = nullptr;
  (void)hipMalloc(&d, (size_t)blocks * 256 * 4);
  std::vector<uint32_t> r0, r1, r2, r3;
  run<Plain>("plain", d, blocks, reps, r0);
  run<Mad64>("mad64", d, blocks, reps, r1);
  run<U24>("u24", d, blocks, reps, r2);
  run<U16>("u16", d, blocks, reps, r3);
  printf("results equal: mad64 %d u24 %d u16 %d\n", (int)(r1 == r0), (int)(r2 == r0), (int)(r3 == r0));
  return 0;
}
