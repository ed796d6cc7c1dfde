// yk_stamps.hpp — the phase-split diagnostic build of the render kernel (tools/phases.py).
//
// With -DYK_STAMPS=1 (make -C uecraytracing_amd/csrc stamps → lib/abl/libykgpu_stamps.so) every
// wave stamps s_memtime at the loop's reconvergence points and sums the cycles per phase into
// the counters ykgpu_get_stats reports as phase_cycles (refill, sample start, interior nodes,
// candidates, shading, path end, leaves; [7] = wave-level node-loop iterations), the first
// wave start / first exhausted claim / last wave exit as timeline, and leaf tests with
// disc >= 0 as diag[0].  The stamps cost ~11% of the wave-cycles and change no result.  In the
// production build every macro below is empty.
#pragma once

#ifndef YK_STAMPS
#define YK_STAMPS 0
#endif

#if YK_STAMPS
#define YK_STAMPS_BEGIN(counters, lane)                                                           \
  uint64_t st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};                                                  \
  uint64_t st_diag0 = 0;                                                                          \
  uint64_t st_prev = __builtin_amdgcn_s_memtime();                                                \
  if ((lane) == 0) atomicMin(&(counters)[16], (unsigned long long)__builtin_amdgcn_s_memrealtime())
#define YK_STAMPS_EXHAUSTED(counters) \
  atomicMin(&(counters)[17], (unsigned long long)__builtin_amdgcn_s_memrealtime())
#define YK_STAMP(k)                                                                  \
  do {                                                                               \
    uint64_t t_;                                                                     \
    __builtin_amdgcn_sched_barrier(0);                                               \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");       \
    __builtin_amdgcn_sched_barrier(0);                                               \
    st_acc[k] += t_ - st_prev;                                                       \
    st_prev = t_;                                                                    \
  } while (0)
// wave-level iterations of the interior-node loop: the first active lane counts
#define YK_STAMP_NODE_ITERATION(lane) \
  do {                                \
    if ((uint32_t)__builtin_ctzll(__ballot(1)) == (lane)) ++st_acc[7]; \
  } while (0)
#define YK_STAMP_DISC_POS() ++st_diag0
#define YK_STAMPS_END(counters, lane)                                                               \
  do {                                                                                              \
    if ((lane) == 0)                                                                                \
      for (int k_ = 0; k_ < 7; ++k_) atomicAdd(&(counters)[8 + k_], (unsigned long long)st_acc[k_]); \
    atomicAdd(&(counters)[15], (unsigned long long)st_acc[7]);                                      \
    atomicAdd(&(counters)[19], (unsigned long long)st_diag0);                                       \
    if ((lane) == 0) atomicMax(&(counters)[18], (unsigned long long)__builtin_amdgcn_s_memrealtime()); \
  } while (0)
#else
#define YK_STAMPS_BEGIN(counters, lane) \
  do {                                  \
  } while (0)
#define YK_STAMPS_EXHAUSTED(counters) \
  do {                                \
  } while (0)
#define YK_STAMP(k) \
  do {              \
  } while (0)
#define YK_STAMP_NODE_ITERATION(lane) \
  do {                                \
  } while (0)
#define YK_STAMP_DISC_POS() \
  do {                      \
  } while (0)
#define YK_STAMPS_END(counters, lane) \
  do {                                \
  } while (0)
#endif
