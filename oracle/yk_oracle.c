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

typedef struct {
  uint32_t x[MT_N];
  uint32_t p;
  uint64_t draws;
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
  if (g->p >= MT_N) mt_twist(g);
  uint32_t z = g->x[g->p++];
  z ^= (z >> 11);
  z ^= (z << 7) & 0x9d2c5680u;
  z ^= (z << 15) & 0xefc60000u;
  z ^= (z >> 18);
  g->draws++;
  return z;
}

/* generate_canonical<double, 53>: random.hpp:161-183.  r = 2^32, so m = 2 draws:
 * sum = u0*1 + u1*2^32 (one rounding in the second add), ret = sum / 2^64, clamped below 1. */
static double mt_canonical(mt_t* g) {
  double sum = 0.0, tmp = 1.0;
  sum += (double)mt_next(g) * tmp;
  tmp *= 4294967296.0;
  sum += (double)mt_next(g) * tmp;
  tmp *= 4294967296.0;
  double ret = sum / tmp;
  if (ret >= 1.0) ret = 1.0 - 0x1p-53; /* 1 - epsilon/2 */
  return ret;
}

/* uniform_real_distribution<double>::operator(): random.hpp:273-278: c*(b-a)+a */
static double mt_uniform(mt_t* g, double a, double b) { return (mt_canonical(g) * (b - a)) + a; }

/* ------------------------------------------------------------------ math.hpp:10-19 */
static double nsqrt(double s) {
  double x = s / 2.0, prev = 0.0;
  int guard = 0; /* never reached for finite s; keeps a NaN input from spinning forever */
  while (x != prev && guard++ < 4096) {
    prev = x;
    x = (x + s / x) / 2.0;
  }
  return x;
}

/* ------------------------------------------------------------------ vec3 helpers (vec3.hpp) */
typedef struct { double x, y, z; } v3;
static inline v3 v3_add(v3 a, v3 b) { v3 r = {a.x + b.x, a.y + b.y, a.z + b.z}; return r; }
static inline v3 v3_sub(v3 a, v3 b) { v3 r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }
static inline v3 v3_mul(v3 a, double s) { v3 r = {a.x * s, a.y * s, a.z * s}; return r; }
static inline v3 v3_div(v3 a, double s) { v3 r = {a.x / s, a.y / s, a.z / s}; return r; }
static inline v3 v3_neg(v3 a) { v3 r = {-a.x, -a.y, -a.z}; return r; }
static inline double v3_dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; } /* :145-147 */
static inline double v3_len2(v3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }      /* :129 */
static inline v3 v3_normalized(v3 a) { return v3_div(a, nsqrt(v3_len2(a))); }        /* :127,132 */
/* near_zero, vec3.hpp:76-80 — note the reference tests x twice and never z */
static inline int v3_near_zero(v3 a) {
  double ax = a.x > 0 ? a.x : -a.x, ay = a.y > 0 ? a.y : -a.y;
  return (ax < 1e-8) && (ay < 1e-8) && (ax < 1e-8);
}
/* reflect, vec3.hpp:199-202: v - 2*dot(v,n)*n */
static inline v3 v3_reflect(v3 v, v3 n) { return v3_sub(v, v3_mul(n, 2 * v3_dot(v, n))); }
static inline v3 v3_of(const double* p) { v3 r = {p[0], p[1], p[2]}; return r; }

/* vec3::random(gen, -1, 1): vec3.hpp:134-142, x then y then z */
static inline v3 v3_random(mt_t* g, double lo, double hi) {
  v3 r;
  r.x = mt_uniform(g, lo, hi);
  r.y = mt_uniform(g, lo, hi);
  r.z = mt_uniform(g, lo, hi);
  return r;
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

typedef struct {
  v3 p, normal;
  double t;
  uint32_t id;
  int front_face;
} hit_t;

/* sphere::hit_impl, sphere.hpp:25-48; set_face_normal, hittable.hpp:23-27 */
static int sphere_hit(const yk_sphere* sp, v3 o, v3 d, double t_min, double t_max, hit_t* rec) {
  v3 c = v3_of(sp->center);
  v3 oc = v3_sub(o, c);
  double a = v3_len2(d);
  double half_b = v3_dot(oc, d);
  double cc = v3_len2(oc) - sp->radius * sp->radius;
  double disc = half_b * half_b - a * cc;
  if (disc < 0) return 0;
  double sq = nsqrt(disc);
  double root = (-half_b - sq) / a;
  if (root < t_min || t_max < root) {
    root = (-half_b + sq) / a;
    if (root < t_min || t_max < root) return 0;
  }
  rec->t = root;
  rec->p = v3_add(o, v3_mul(d, root)); /* ray::at, ray.hpp:16-19 */
  v3 outward = v3_div(v3_sub(rec->p, c), sp->radius);
  rec->front_face = v3_dot(d, outward) < 0;
  rec->normal = rec->front_face ? outward : v3_neg(outward);
  return 1;
}

/* hittable_list::hit_impl, hittable_list.hpp:32-58: ordered scan, shrinking closest_so_far,
 * the last accepted object (= closest, ties to the later index) wins. */
static int world_hit(world_t* w, v3 o, v3 d, double t_min, double t_max, hit_t* out) {
  double closest = t_max;
  int any = 0;
  hit_t tmp;
  for (uint32_t i = 0; i < w->n; ++i) {
    w->tests++;
    if (sphere_hit(&w->s[i], o, d, t_min, closest, &tmp)) {
      closest = tmp.t;
      tmp.id = i;
      *out = tmp;
      any = 1;
    }
  }
  return any;
}

/* Schlick, RTIOW (extension) — (1-c)^5 as an explicit left-to-right product */
static double reflectance(double cosine, double ref_idx) {
  double r0 = (1 - ref_idx) / (1 + ref_idx);
  r0 = r0 * r0;
  double x = 1 - cosine;
  return r0 + (1 - r0) * ((((x * x) * x) * x) * x);
}

/* scatter dispatch hittable_list.hpp:60-73 → sphere.hpp:50-54 → material.hpp */
static int scatter(const yk_sphere* sp, v3 rd, const hit_t* rec, mt_t* g, c3* att, v3* dir) {
  switch (sp->material) {
    case YK_MATERIAL_LAMBERTIAN: { /* material.hpp:50-59, random_unit_vector :33-36 */
      v3 ru = v3_random(g, -1, 1);
      ru = v3_div(ru, nsqrt(v3_len2(ru))); /* normalize(): *this /= length() */
      v3 sd = v3_add(rec->normal, ru);
      if (v3_near_zero(sd)) sd = rec->normal;
      *dir = sd;
      att->r = sp->albedo[0]; att->g = sp->albedo[1]; att->b = sp->albedo[2];
      return 1;
    }
    case YK_MATERIAL_METAL: { /* material.hpp:67-75 (+ fuzz extension) */
      v3 refl = v3_reflect(v3_normalized(rd), rec->normal);
      if (sp->fuzz > 0) { /* extension: random_in_unit_sphere, material.hpp:27-30 */
        v3 ru = v3_random(g, -1, 1);
        ru = v3_div(ru, nsqrt(v3_len2(ru)));
        double k = mt_uniform(g, 0.01, 0.99);
        refl = v3_add(refl, v3_mul(v3_mul(ru, k), sp->fuzz));
      }
      if (v3_dot(refl, rec->normal) > 0) {
        *dir = refl;
        att->r = sp->albedo[0]; att->g = sp->albedo[1]; att->b = sp->albedo[2];
        return 1;
      }
      return 0;
    }
    case YK_MATERIAL_DIELECTRIC: { /* extension (RTIOW dielectric, yk-style arithmetic) */
      double ratio = rec->front_face ? (1.0 / sp->ior) : sp->ior;
      v3 unit = v3_normalized(rd);
      double ct = v3_dot(v3_neg(unit), rec->normal);
      if (!(ct < 1.0)) ct = 1.0;
      double st = nsqrt(1.0 - ct * ct);
      int cannot = ratio * st > 1.0;
      if (cannot || reflectance(ct, ratio) > mt_uniform(g, 0, 1)) {
        *dir = v3_reflect(unit, rec->normal);
      } else {
        v3 perp = v3_mul(v3_add(unit, v3_mul(rec->normal, ct)), ratio);
        double pl = 1.0 - v3_len2(perp);
        v3 par = v3_mul(rec->normal, -nsqrt(pl < 0 ? -pl : pl));
        *dir = v3_add(perp, par);
      }
      att->r = 1.0; att->g = 1.0; att->b = 1.0;
      return 1;
    }
  }
  return 0;
}

/* raytracer::ray_color, raytracer.hpp:19-37 — kept recursive, exactly like the reference */
static c3 ray_color(world_t* w, v3 o, v3 d, uint32_t depth, mt_t* g, uint64_t* segs) {
  c3 black = {0, 0, 0};
  if (depth == 0) return black;
  hit_t rec;
  if (segs) (*segs)++;
  if (world_hit(w, o, d, w->p->t_min, INFINITY, &rec)) {
    c3 att;
    v3 nd;
    if (scatter(&w->s[rec.id], d, &rec, g, &att, &nd)) {
      c3 in = ray_color(w, rec.p, nd, depth - 1, g, segs);
      c3 r = {att.r * in.r, att.g * in.g, att.b * in.b};
      return r;
    }
    return black;
  }
  double t = (v3_normalized(d).y + 1.0) / 2;
  c3 r = {(1.0 - t) * 1.0 + t * 0.5, (1.0 - t) * 1.0 + t * 0.7, (1.0 - t) * 1.0 + t * 1.0};
  return r;
}

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

/* One sample: source.cpp:154-166 (seed :154-158, jitter :160-164, get_ray camera.hpp:29-32
 * or the thin-lens extension). */
static c3 sample(world_t* w, uint32_t y, uint32_t x, uint32_t s, uint64_t* draws, uint64_t* segs) {
  const yk_render_params* p = w->p;
  const yk_camera* cam = w->cam;
  mt_t g;
  uint32_t seed = p->seed0 + (y * p->image_width + x) * p->samples_per_pixel + s;
  if (w->as_shipped) seed = random_device_u32();
  mt_seed(&g, seed);
  double u = (x + mt_uniform(&g, 0, 1)) / p->image_width;
  double v = (p->image_height - y - 1 + mt_uniform(&g, 0, 1)) / p->image_height;
  v3 org = v3_of(cam->origin);
  v3 dir = v3_add(v3_add(v3_of(cam->lower_left_corner), v3_mul(v3_of(cam->horizontal), u)),
                  v3_mul(v3_of(cam->vertical), v));
  dir = v3_sub(dir, org);
  if (cam->lens_radius > 0) { /* extension: random_in_unit_disk by rejection */
    double px, py;
    for (;;) {
      px = mt_uniform(&g, -1, 1);
      py = mt_uniform(&g, -1, 1);
      if (px * px + py * py < 1.0) break;
    }
    double rx = px * cam->lens_radius, ry = py * cam->lens_radius;
    v3 off = v3_add(v3_mul(v3_of(cam->lens_u), rx), v3_mul(v3_of(cam->lens_v), ry));
    org = v3_add(org, off);
    dir = v3_sub(dir, off);
  }
  c3 c = ray_color(w, org, dir, p->max_depth, &g, segs);
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

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  world_t w = {j->s, j->n, j->cam, j->p, 0, j->as_shipped};
  const uint32_t W = j->p->image_width;
  for (uint32_t i = j->tid; i < j->p->row_count; i += j->nthreads) {
    uint32_t y = j->p->row_begin + i * j->p->row_stride;
    for (uint32_t x = 0; x < W; ++x) {
      c3 ps = pixel_sum(&w, y, x, &j->segs);
      size_t o = ((size_t)i * W + x) * 3;
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
  if (p->row_count && (p->row_stride == 0 ||
      (uint64_t)p->row_begin + (uint64_t)(p->row_count - 1) * p->row_stride >= p->image_height))
    return YK_ERR_INVALID;
  if (p->precision != YK_PRECISION_FP64 || p->rng != YK_RNG_MT19937) return YK_ERR_UNSUPPORTED;
  return YK_OK;
}

/* ------------------------------------------------------------------ exported (ctypes) */

/* Render the rows named by p into rgb (row_count*W*3 bytes) and/or sums (row_count*W*3
 * doubles), with `nthreads` host threads over interleaved rows.  Returns YK_* status;
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
