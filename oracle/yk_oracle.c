/*
 * oracle/yk_oracle.c — TEST INFRASTRUCTURE ONLY.
 *
 * A plain-C, CPU restatement of the reference's per-pixel sampling loop, used as the parity
 * checker for the HIP path and as the `cpu_baseline` ("port") of bench.py.  It is never linked
 * into, loaded by or called from the product (uecraytracing_amd/); only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg load it (oracle/_build/libykoracle.so).
 *
 * Pinned: tests/test_oracle_golden.py checks it byte-for-byte / bit-for-bit against fixtures
 * generated from the reference itself (oracle/ref_harness.cpp compiled against
 * /root/reference/yk/*.hpp; tests/golden/gen_golden.py), for the reference's materials and
 * camera.  The extensions (metal fuzz, dielectric, thin-lens camera; BASELINE configs 2-5) have
 * no reference code: their parity is UNPINNED and holds only between this file and the GPU.
 *
 * Everything is deliberately written the obvious, scalar, recursive way, mirroring the
 * reference's evaluation order operation by operation (no FMA contraction: build with
 * -ffp-contract=off).  Citations are /root/reference/<file>:<line>.
 */
#include <math.h>
#include <fcntl.h>
#include <pthread.h>
#include <unistd.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/ykgpu.h"

/* ------------------------------------------------------------------ mt19937 (random.hpp) */
#define MT_N 624
#define MT_M 397

/* The per-sample engine: mt19937 (the reference's, random.hpp:43-151) or, for YK_RNG_XOR128,
 * the reference's other engine yk::xor128 (random.hpp:18-41) in xs[]. */
typedef struct {
  uint32_t x[MT_N];
  uint32_t p;
  uint64_t draws;
  uint32_t kind; /* YK_RNG_* */
  uint32_t xs[4];
} mt_t;

/* seed(): random.hpp:69-81 (x_i = 1812433253 * (x_{i-1} ^ x_{i-1} >> 30) + i, mod 2^32) */
static void mt_seed(mt_t* g, uint32_t sd) {
  g->x[0] = sd;
  for (uint32_t i = 1; i < MT_N; ++i) {
    uint32_t v = g->x[i - 1];
    v ^= v >> 30;
    g->x[i] = v * 1812433253u + i;
  }
  g->p = MT_N;
  g->draws = 0;
  g->kind = YK_RNG_MT19937;
}

/* xor128(seed): x, y, z at their default member values, w = 88675123 ^ seed (random.hpp:19-32) */
static void x128_seed(mt_t* g, uint32_t sd) {
  g->xs[0] = 123456789u;
  g->xs[1] = 362436069u;
  g->xs[2] = 521288629u;
  g->xs[3] = 88675123u ^ sd;
  g->draws = 0;
  g->kind = YK_RNG_XOR128;
}

static void rng_seed(mt_t* g, uint32_t sd, uint32_t kind) {
  if (kind == YK_RNG_XOR128) x128_seed(g, sd);
  else mt_seed(g, sd);
}

static inline uint32_t mt_mix(uint32_t hi_src, uint32_t lo_src) {
  uint32_t y = (hi_src & 0x80000000u) | (lo_src & 0x7fffffffu);
  return (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}

/* M_gen_rand(): random.hpp:114-131 */
static void mt_twist(mt_t* g) {
  uint32_t k;
  for (k = 0; k < MT_N - MT_M; ++k) g->x[k] = g->x[k + MT_M] ^ mt_mix(g->x[k], g->x[k + 1]);
  for (; k < MT_N - 1; ++k) g->x[k] = g->x[k + MT_M - MT_N] ^ mt_mix(g->x[k], g->x[k + 1]);
  g->x[MT_N - 1] = g->x[MT_M - 1] ^ mt_mix(g->x[MT_N - 1], g->x[0]);
  g->p = 0;
}

/* operator(): random.hpp:95-105 (tempering) */
static uint32_t mt_next(mt_t* g) {
  if (g->kind == YK_RNG_XOR128) { /* xor128::operator(), random.hpp:34-40 */
    uint32_t t = g->xs[0] ^ (g->xs[0] << 11);
    g->xs[0] = g->xs[1];
    g->xs[1] = g->xs[2];
    g->xs[2] = g->xs[3];
    g->xs[3] = (g->xs[3] ^ (g->xs[3] >> 19)) ^ (t ^ (t >> 8));
    g->draws++;
    return g->xs[3];
  }
  if (g->p >= MT_N) mt_twist(g);
  uint32_t z = g->x[g->p++];
  z ^= (z >> 11);
  z ^= (z << 7) & 0x9d2c5680u;
  z ^= (z << 15) & 0xefc60000u;
  z ^= (z >> 18);
  g->draws++;
  return z;
}

typedef struct { double r, g, b; } c3;

/* ------------------------------------------------------------------ scene */
typedef struct {
  const yk_sphere* s;
  uint32_t n;
  const yk_camera* cam;
  const yk_render_params* p;
  uint64_t tests; /* ray-sphere tests (diagnostics) */
  int as_shipped; /* seed every sample from /dev/urandom like the runtime build (timing only) */
} world_t;

/* ------------------------------------------------------------------ the path, per real type */
static const double kEps_d = 0x1p-52; /* numeric_limits<double>::epsilon() */
static const float kEps_f = 0x1p-23f; /* numeric_limits<float>::epsilon()  */

#define R double
#define SFX(name) name##_d
#define YKO_CANON_DRAWS 2
#include "yk_oracle_path.h"
#undef R
#undef SFX
#undef YKO_CANON_DRAWS

#define R float
#define SFX(name) name##_f
#define YKO_CANON_DRAWS 1
#include "yk_oracle_path.h"
#undef R
#undef SFX
#undef YKO_CANON_DRAWS

/* the double names the rest of this file (and its KAT exports) use */
#define mt_uniform uniform_d
#define nsqrt nsqrt_d

/* The runtime build's seed, source.cpp:159: a std::random_device constructed per sample.
 * libstdc++'s random_device opens its entropy source, reads one word and closes it again; this
 * models that cost with /dev/urandom (timing of the as-shipped cost model only: the image is not
 * reproducible, as in the reference). */
static uint32_t random_device_u32(void) {
  uint32_t v = 0;
  int fd = open("/dev/urandom", O_RDONLY);
  if (fd >= 0) {
    if (read(fd, &v, sizeof v) != (ssize_t)sizeof v) v = 0;
    close(fd);
  }
  return v;
}

/* YK_SEED_RANDOM_DEVICE: the runtime build gives every sample its own std::random_device seed
 * (source.cpp:159).  The GPU cannot read an entropy device per sample, so the mode hashes one
 * 64-bit key per call with the sample's linear index (splitmix64 finaliser, high word): seeds
 * independent across samples, reproducible given the key (include/ykgpu.h). */
static uint32_t seed_from_key(uint64_t key, uint64_t idx) {
  uint64_t z = key + (idx + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (uint32_t)(z >> 32);
}

/* One sample: source.cpp:154-166 (seed :154-158, then trace_sample in the call's precision). */
static c3 sample(world_t* w, uint32_t y, uint32_t x, uint32_t s, uint64_t* draws, uint64_t* segs) {
  const yk_render_params* p = w->p;
  mt_t g;
  uint32_t seed = p->seed0 + (y * p->image_width + x) * p->samples_per_pixel + s;
  if (p->seed_mode == YK_SEED_RANDOM_DEVICE)
    seed = seed_from_key(p->seed_key, ((uint64_t)y * p->image_width + x) * p->samples_per_pixel + s);
  if (w->as_shipped) seed = random_device_u32();
  rng_seed(&g, seed, p->rng);
  c3 c = p->precision == YK_PRECISION_FP32 ? trace_sample_f(w, &g, y, x, segs)
                                           : trace_sample_d(w, &g, y, x, segs);
  if (draws) *draws = g.draws;
  return c;
}

/* transform_reduce over iota(0, spp) (source.cpp:137-167).  libstdc++'s transform_reduce
 * (/usr/include/c++/11/numeric:437-461) only takes its group-of-4 branch for iterators whose
 * iterator_traits category is random access; iota_view's iterator reports
 * input_iterator_tag (its reference is a prvalue), so the reference sums strictly
 * sequentially: init = ((0 + c0) + c1) + ... (pinned by the golden per-pixel sums). */
static c3 pixel_sum(world_t* w, uint32_t y, uint32_t x, uint64_t* segs) {
  c3 init = {0, 0, 0};
  for (uint32_t s = 0; s < w->p->samples_per_pixel; ++s) {
    c3 a = sample(w, y, x, s, 0, segs);
    init.r = init.r + a.r;
    init.g = init.g + a.g;
    init.b = init.b + a.b;
  }
  return init;
}

/* to_color3b, source.cpp:73-83; std::clamp then static_cast<uint8_t> (truncation) */
static uint8_t quantise(double sum, uint32_t spp) {
  double v = nsqrt(sum / spp);
  v = (v < 0.0) ? 0.0 : (0.999 < v) ? 0.999 : v;
  return (uint8_t)(v * 256);
}

typedef struct {
  const yk_sphere* s;
  uint32_t n;
  const yk_camera* cam;
  const yk_render_params* p;
  uint8_t* rgb;
  double* sums;
  uint32_t tid, nthreads;
  uint64_t segs, tests;
  int as_shipped;
} job_t;

/* Image row of tile row i of the row set (include/ykgpu.h: bands of 2^row_band_log2 rows, every
 * row_stride-th band; 0 = single rows) */
static uint64_t row_y(const yk_render_params* p, uint32_t i) {
  const uint32_t L = p->row_band_log2;
  return (uint64_t)p->row_begin + ((((uint64_t)(i >> L)) * p->row_stride) << L) + (i & ((1u << L) - 1u));
}

/* ... and image column of tile column c of the column set (ABI 10: col_count == 0 = every
 * column; else bands of 2^col_band_log2 columns, every col_stride-th band) */
static uint32_t tile_w(const yk_render_params* p) { return p->col_count ? p->col_count : p->image_width; }
static uint64_t col_x(const yk_render_params* p, uint32_t c) {
  if (!p->col_count) return c;
  const uint32_t L = p->col_band_log2;
  return (uint64_t)p->col_begin + ((((uint64_t)(c >> L)) * p->col_stride) << L) + (c & ((1u << L) - 1u));
}

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  world_t w = {j->s, j->n, j->cam, j->p, 0, j->as_shipped};
  const uint32_t Wt = tile_w(j->p);
  /* pixels dealt to the threads one by one (a single row still uses every thread) */
  const uint64_t npix = (uint64_t)j->p->row_count * Wt;
  for (uint64_t k = j->tid; k < npix; k += j->nthreads) {
    const uint32_t i = (uint32_t)(k / Wt), c = (uint32_t)(k % Wt);
    const uint32_t y = (uint32_t)row_y(j->p, i), x = (uint32_t)col_x(j->p, c);
    {
      c3 ps = pixel_sum(&w, y, x, &j->segs);
      size_t o = ((size_t)i * Wt + c) * 3;
      if (j->sums) { j->sums[o] = ps.r; j->sums[o + 1] = ps.g; j->sums[o + 2] = ps.b; }
      if (j->rgb) {
        j->rgb[o] = quantise(ps.r, j->p->samples_per_pixel);
        j->rgb[o + 1] = quantise(ps.g, j->p->samples_per_pixel);
        j->rgb[o + 2] = quantise(ps.b, j->p->samples_per_pixel);
      }
    }
  }
  j->tests = w.tests;
  return 0;
}

static int check(const yk_sphere* s, uint32_t n, const yk_camera* cam, const yk_render_params* p) {
  if (!s || !n || !cam || !p) return YK_ERR_INVALID;
  if (!p->image_width || !p->image_height || !p->samples_per_pixel) return YK_ERR_INVALID;
  if (p->row_count && (p->row_stride == 0 || p->row_band_log2 > 10 ||
      row_y(p, p->row_count - 1) >= p->image_height))
    return YK_ERR_INVALID;
  if (p->col_count ? (p->col_stride == 0 || p->col_band_log2 > 10 || col_x(p, p->col_count - 1) >= p->image_width)
                   : (p->col_begin || p->col_stride || p->col_band_log2))
    return YK_ERR_INVALID;
  if ((p->precision != YK_PRECISION_FP64 && p->precision != YK_PRECISION_FP32) || (p->rng != YK_RNG_MT19937 && p->rng != YK_RNG_XOR128) ||
      p->seed_mode > YK_SEED_RANDOM_DEVICE || (p->seed_mode == YK_SEED_RANDOM_DEVICE && !p->seed_key))
    return YK_ERR_UNSUPPORTED;
  return YK_OK;
}

/* ------------------------------------------------------------------ exported (ctypes) */

/* Render the tile named by p (its rows, and its columns when col_count > 0) into rgb
 * (row_count*Wt*3 bytes) and/or sums (row_count*Wt*3 doubles), with `nthreads` host threads over interleaved pixels.  Returns YK_* status;
 * *segments / *tests (nullable) receive work counts. */
static int render_impl(const yk_sphere* s, uint32_t n, const yk_camera* cam, const yk_render_params* p,
                       uint8_t* rgb, double* sums, int nthreads, uint64_t* segments, uint64_t* tests,
                       int as_shipped) {
  int st = check(s, n, cam, p);
  if (st) return st;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  job_t* jobs = (job_t*)calloc((size_t)nthreads, sizeof(job_t));
  pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
  if (!jobs || !th) { free(jobs); free(th); return YK_ERR_NOMEM; }
  for (int t = 0; t < nthreads; ++t) {
    job_t jj = {s, n, cam, p, rgb, sums, (uint32_t)t, (uint32_t)nthreads, 0, 0, as_shipped};
    jobs[t] = jj;
  }
  for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], 0, worker, &jobs[t]);
  worker(&jobs[0]);
  uint64_t sg = jobs[0].segs, ts = jobs[0].tests;
  for (int t = 1; t < nthreads; ++t) {
    pthread_join(th[t], 0);
    sg += jobs[t].segs;
    ts += jobs[t].tests;
  }
  if (segments) *segments = sg;
  if (tests) *tests = ts;
  free(jobs);
  free(th);
  return YK_OK;
}

int yko_render(const yk_sphere* s, uint32_t n, const yk_camera* cam, const yk_render_params* p,
               uint8_t* rgb, double* sums, int nthreads, uint64_t* segments, uint64_t* tests) {
  return render_impl(s, n, cam, p, rgb, sums, nthreads, segments, tests, 0);
}

/* The same loop with the runtime build's per-sample random_device seeding (source.cpp:159): the
 * reference's as-shipped cost model for the CPU baseline (SURVEY §8(d) variant i).  Timing only. */
int yko_render_as_shipped(const yk_sphere* s, uint32_t n, const yk_camera* cam, const yk_render_params* p,
                          uint8_t* rgb, double* sums, int nthreads, uint64_t* segments, uint64_t* tests) {
  return render_impl(s, n, cam, p, rgb, sums, nthreads, segments, tests, 1);
}

/* One sample's colour and its u32 draw count (per-sample path fixtures). */
int yko_sample(const yk_sphere* s, uint32_t n, const yk_camera* cam, const yk_render_params* p,
               uint32_t y, uint32_t x, uint32_t smp, double* rgb3, uint64_t* draws) {
  int st = check(s, n, cam, p);
  if (st) return st;
  world_t w = {s, n, cam, p, 0, 0};
  c3 c = sample(&w, y, x, smp, draws, 0);
  rgb3[0] = c.r; rgb3[1] = c.g; rgb3[2] = c.b;
  return YK_OK;
}

/* First `count` mt19937 outputs for `seed`. */
void yko_mt19937(uint32_t seed, uint32_t count, uint32_t* out) {
  mt_t g;
  mt_seed(&g, seed);
  for (uint32_t i = 0; i < count; ++i) out[i] = mt_next(&g);
}

/* The ref_harness KAT pattern: canonical (0,1) twice, then uniform(-1,1), repeated. */
void yko_canonical_pattern(uint32_t seed, uint32_t count, double* out) {
  mt_t g;
  mt_seed(&g, seed);
  for (uint32_t i = 0; i < count; ++i) out[i] = (i % 3 == 2) ? mt_uniform(&g, -1, 1) : mt_uniform(&g, 0, 1);
}

double yko_newton_sqrt(double s) { return nsqrt(s); }

/* Same over an array (the GPU test of ykgpu_math_sqrt).  Inputs must be finite and >= 0: the
 * reference's loop never ends for NaN, inf or negative s. */
void yko_newton_sqrt_n(const double* in, double* out, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) out[i] = nsqrt(in[i]);
}

/* FP32 path (render<float>): the KAT pattern with uniform_real_distribution<float> (one draw per
 * canonical), and math::sqrt<float> over an array. */
void yko_canonical_pattern_f32(uint32_t seed, uint32_t count, float* out) {
  mt_t g;
  mt_seed(&g, seed);
  for (uint32_t i = 0; i < count; ++i) out[i] = (i % 3 == 2) ? uniform_f(&g, -1, 1) : uniform_f(&g, 0, 1);
}

void yko_newton_sqrt_f32_n(const float* in, float* out, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) out[i] = nsqrt_f(in[i]);
}

/* The per-sample seed of YK_SEED_RANDOM_DEVICE (include/ykgpu.h), for tests. */
uint32_t yko_seed_from_key(uint64_t key, uint64_t idx) { return seed_from_key(key, idx); }

/* First `count` xor128 outputs for `seed` (random.hpp:18-41), and the KAT canonical pattern. */
void yko_xor128(uint32_t seed, uint32_t count, uint32_t* out) {
  mt_t g;
  x128_seed(&g, seed);
  for (uint32_t i = 0; i < count; ++i) out[i] = mt_next(&g);
}

void yko_canonical_pattern_x128(uint32_t seed, uint32_t count, double* out) {
  mt_t g;
  x128_seed(&g, seed);
  for (uint32_t i = 0; i < count; ++i) out[i] = (i % 3 == 2) ? mt_uniform(&g, -1, 1) : mt_uniform(&g, 0, 1);
}
