// tools/ldsbench.hip — does an LDS read cost LDS cycles for lanes the exec mask turns off?
// Each wave runs a chain of dependent ds_read_b128 (the next address comes from the data read)
// plus independent ones, with K of its 64 lanes active; waves per CU as the render's (12).  If the
// time per read stays flat as K drops, masked lanes are free in the LDS pipe and only the latency
// matters; if it scales with K, the LDS is bandwidth-bound on active lanes only.
//   build: hipcc -O3 --offload-arch=gfx950 -o tools/ldsbench tools/ldsbench.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s\n", hipGetErrorString(e_)); return 1; } } while (0)

constexpr int kLdsWords = 8192;  // 32 KB of uint4-addressable table
template <int kIndep>
__global__ __launch_bounds__(768) void lds_chain(int active, int iters, unsigned* out) {
  __shared__ uint4 tab[kLdsWords / 4];
  for (int i = threadIdx.x; i < kLdsWords / 4; i += blockDim.x)
    tab[i] = make_uint4((i * 7 + 1) % (kLdsWords / 4), i, i ^ 5, i + 3);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  unsigned acc = 0;
  if (lane < active) {
    unsigned idx = (threadIdx.x * 13) % (kLdsWords / 4);
    for (int it = 0; it < iters; ++it) {
      const uint4 v = tab[idx];
      acc += v.y;
#pragma unroll
      for (int k = 0; k < kIndep; ++k) {
        const uint4 w = tab[(idx + 37 * (k + 1)) % (kLdsWords / 4)];
        acc ^= w.z;
      }
      idx = v.x;
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  int dev = 0;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, dev));
  unsigned* out;
  CHECK(hipMalloc(&out, 4));
  const int cus = prop.multiProcessorCount, iters = 4096;
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  printf("{\"device\": \"%s\", \"cus\": %d}\n", prop.gcnArchName, cus);
  for (int indep : {0, 6}) {
    for (int active : {64, 32, 16, 8, 1}) {
      for (int rep = 0; rep < 2; ++rep) {
        CHECK(hipEventRecord(a));
        if (indep == 0)
          hipLaunchKernelGGL(lds_chain<0>, dim3(cus), dim3(768), 0, 0, active, iters, out);
        else
          hipLaunchKernelGGL(lds_chain<6>, dim3(cus), dim3(768), 0, 0, active, iters, out);
        CHECK(hipEventRecord(b));
        CHECK(hipEventSynchronize(b));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, a, b));
        if (rep == 1) {
          const double reads = (double)iters * (1 + indep);
          const double cyc = ms * 1e-3 * prop.clockRate * 1e3 / reads;  // per read, per wave (12 waves/CU)
          printf("{\"reads_per_iter\": %d, \"active_lanes\": %d, \"ms\": %.4f, \"cu_cycles_per_read_round\": %.2f}\n",
                 1 + indep, active, ms, cyc);
        }
      }
    }
  }
  return 0;
}
