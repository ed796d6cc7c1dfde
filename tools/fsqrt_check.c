/* tools/fsqrt_check.c — exhaustive check behind the FP32 path's math::sqrt<float>
 * (uecraytracing_amd/csrc/yk_device_f32.hpp).
 *
 * For every positive finite float s: (1) the reference loop of math.hpp:10-19 with T = float
 * (x = s / 2.0; x = (x + s / x) / 2.0 until x == prev; halving in double, as the literal 2.0
 * makes it) terminates, and (2) the same iteration started at the correctly rounded sqrtf(s)
 * ends at the same float.  Prints the number of hangs, of differing results (and of those
 * inside [2^-100, 2^100], the range where the GPU uses the sqrtf start) and the largest
 * iteration count; and (3) that ONE step from sqrtf(s), (r + s/r) * 0.5f, already equals the loop's
 * result inside [2^-100, 2^100] (the device's form).  Measured: hang 0, diff 1,
 * diff_in[2^-100,2^100] 0, maxit 80, onestep_diff_in[2^-100,2^100] 0 (~2 min, 8 threads).
 *
 *   gcc -O2 -ffp-contract=off -o /tmp/fsqrt_check tools/fsqrt_check.c -lpthread -lm
 */
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <math.h>
#include <pthread.h>
/* math.hpp:10-19 with T=float */
static int ref(float s, float* out) {
  float x = (float)((double)s / 2.0), prev = 0.0f; int it = 0;
  while (x != prev) { prev = x; x = (float)((double)(x + s / x) / 2.0); if (++it > 2000) return -1; }
  *out = x; return it;
}
static int from(float s, float x0, float* out) {
  float x = x0, prev = 0.0f; int it = 0;
  while (x != prev) { prev = x; x = (x + s / x) * 0.5f; if (++it > 2000) return -1; }
  *out = x; return it;
}
typedef struct { uint32_t lo, hi; uint64_t hang, diff, maxit, diff_small, onestep_diff; uint32_t ex; } job;
static void* run(void* a) {
  job* j = a;
  for (uint32_t b = j->lo; b < j->hi; ++b) {
    float s; memcpy(&s, &b, 4);
    float r1, r2;
    int i1 = ref(s, &r1);
    if (i1 < 0) { j->hang++; j->ex = b; continue; }
    if ((uint64_t)i1 > j->maxit) j->maxit = i1;
    int i2 = from(s, sqrtf(s), &r2);
    if (i2 < 0 || r1 != r2) { if (s >= 0x1p-100f && s <= 0x1p100f) j->diff_small++; j->diff++; }
    /* (3) one step from the correctly rounded sqrtf(s) already lands on the loop's result */
    if (s >= 0x1p-100f && s <= 0x1p100f) {
      const float r = sqrtf(s), x1 = (r + s / r) * 0.5f;
      if (x1 != r1) j->onestep_diff++;
    }
  }
  return 0;
}
int main() {
  /* positive finite floats excluding 0: bits 1 .. 0x7f7fffff */
  const int T = 8; pthread_t th[T]; job jb[T];
  uint32_t N = 0x7f800000u;
  for (int t = 0; t < T; ++t) { jb[t] = (job){1 + (uint64_t)N * t / T, 1 + (uint64_t)N * (t + 1) / T - (t==T-1), 0,0,0,0,0,0}; pthread_create(&th[t], 0, run, &jb[t]); }
  uint64_t hang = 0, diff = 0, maxit = 0, ds = 0, os = 0;
  for (int t = 0; t < T; ++t) { pthread_join(th[t], 0); hang += jb[t].hang; diff += jb[t].diff; ds += jb[t].diff_small; os += jb[t].onestep_diff; if (jb[t].maxit > maxit) maxit = jb[t].maxit; if (jb[t].hang) printf("hang example %08x\n", jb[t].ex);}
  printf("hang %llu diff %llu diff_in[2^-100,2^100] %llu maxit %llu onestep_diff_in[2^-100,2^100] %llu\n", (unsigned long long)hang, (unsigned long long)diff, (unsigned long long)ds, (unsigned long long)maxit, (unsigned long long)os);
}
