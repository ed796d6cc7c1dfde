/*
 * oracle/yk_oracle_path.h — TEST INFRASTRUCTURE ONLY (see yk_oracle.c).
 *
 * The per-sample path of the reference, written once over the real type R and included twice
 * by yk_oracle.c: R = double is render() as shipped (source.cpp:98, T = double); R = float is the
 * same template instantiated with T = float (YK_PRECISION_FP32).  Colours stay double in both
 * (raytracer<T, double>, lambertian<double>: source.cpp:100,106-111).
 *
 * The text follows C++'s usual arithmetic conversions exactly as the reference's expressions do
 * (C has the same rules): a float operand meeting a double literal is promoted, so e.g.
 * math::sqrt's `s / 2.0` and the sky's `y + 1.0` are double operations for R = float, as in
 * the reference.  Extension code (fuzz, dielectric, thin lens; no reference) uses R literals.
 *
 * Expects: R, SFX(name), YKO_CANON_DRAWS (2 for double, 1 for float), and yk_oracle.c's mt_t,
 * c3, world_t, mt_next.
 */

/* generate_canonical<R, digits>: random.hpp:161-183.  r = 2^32 and log2r = bit_width(2^32) = 33,
 * so m = max(1, (digits + 32) / 33): 2 draws for double, 1 for float.  sum = u0 (+ u1*2^32),
 * ret = sum / 2^(32m) (exact scaling), clamped to 1 - eps/2. */
static R SFX(canonical)(mt_t* g) {
  R sum = 0, tmp = 1;
  sum += (R)mt_next(g) * tmp;
  tmp *= (R)4294967296.0;
#if YKO_CANON_DRAWS == 2
  sum += (R)mt_next(g) * tmp;
  tmp *= (R)4294967296.0;
#endif
  R ret = sum / tmp;
  if (ret >= (R)1) ret = (R)1 - SFX(kEps) / (R)2;
  return ret;
}

/* uniform_real_distribution<R>::operator(): random.hpp:273-278: c*(b-a)+a */
static R SFX(uniform)(mt_t* g, R a, R b) { return (SFX(canonical)(g) * (b - a)) + a; }

/* math::sqrt<R>, math.hpp:10-19 (verbatim arithmetic: s / 2.0 and (...) / 2.0 are double
 * operations also for R = float, then rounded to R by the assignment) */
static R SFX(nsqrt)(R s) {
  R x = s / 2.0, prev = 0.0;
  int guard = 0; /* never reached for finite s >= 0; keeps a NaN input from spinning forever */
  while (x != prev && guard++ < 4096) {
    prev = x;
    x = (x + s / x) / 2.0;
  }
  return x;
}

/* ------------------------------------------------------------------ vec3<R> (vec3.hpp) */
typedef struct { R x, y, z; } SFX(v3);
#define V3 SFX(v3)
static inline V3 SFX(v3_add)(V3 a, V3 b) { V3 r = {a.x + b.x, a.y + b.y, a.z + b.z}; return r; }
static inline V3 SFX(v3_sub)(V3 a, V3 b) { V3 r = {a.x - b.x, a.y - b.y, a.z - b.z}; return r; }
static inline V3 SFX(v3_mul)(V3 a, R s) { V3 r = {a.x * s, a.y * s, a.z * s}; return r; }
static inline V3 SFX(v3_div)(V3 a, R s) { V3 r = {a.x / s, a.y / s, a.z / s}; return r; }
static inline V3 SFX(v3_neg)(V3 a) { V3 r = {-a.x, -a.y, -a.z}; return r; }
static inline R SFX(v3_dot)(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; } /* :145-147 */
static inline R SFX(v3_len2)(V3 a) { return a.x * a.x + a.y * a.y + a.z * a.z; }      /* :129 */
static inline V3 SFX(v3_normalized)(V3 a) { return SFX(v3_div)(a, SFX(nsqrt)(SFX(v3_len2)(a))); } /* :127,132 */
/* near_zero, vec3.hpp:76-80 — the reference tests x twice and never z; s = 1e-8 is a double, so
 * a float component is compared after promotion */
static inline int SFX(v3_near_zero)(V3 a) {
  R ax = a.x > 0 ? a.x : -a.x, ay = a.y > 0 ? a.y : -a.y;
  return (ax < 1e-8) && (ay < 1e-8) && (ax < 1e-8);
}
/* reflect, vec3.hpp:199-202: v - 2*dot(v,n)*n (2 * dot is an R product) */
static inline V3 SFX(v3_reflect)(V3 v, V3 n) { return SFX(v3_sub)(v, SFX(v3_mul)(n, 2 * SFX(v3_dot)(v, n))); }
static inline V3 SFX(v3_of)(const double* p) { V3 r = {(R)p[0], (R)p[1], (R)p[2]}; return r; }

/* vec3<R>::random(gen, -1, 1): vec3.hpp:134-142, x then y then z */
static inline V3 SFX(v3_random)(mt_t* g, R lo, R hi) {
  V3 r;
  r.x = SFX(uniform)(g, lo, hi);
  r.y = SFX(uniform)(g, lo, hi);
  r.z = SFX(uniform)(g, lo, hi);
  return r;
}

typedef struct {
  V3 p, normal;
  R t;
  uint32_t id;
  int front_face;
} SFX(hit_t);
#define HIT SFX(hit_t)

/* sphere::hit_impl, sphere.hpp:25-48; set_face_normal, hittable.hpp:23-27.  Centre and radius
 * are the record's doubles rounded to R (pos3<T>, T radius: sphere.hpp:18-19). */
static int SFX(sphere_hit)(const yk_sphere* sp, V3 o, V3 d, R t_min, R t_max, HIT* rec) {
  V3 c = SFX(v3_of)(sp->center);
  R radius = (R)sp->radius;
  V3 oc = SFX(v3_sub)(o, c);
  R a = SFX(v3_len2)(d);
  R half_b = SFX(v3_dot)(oc, d);
  R cc = SFX(v3_len2)(oc) - radius * radius;
  R disc = half_b * half_b - a * cc;
  if (disc < 0) return 0;
  R sq = SFX(nsqrt)(disc);
  R root = (-half_b - sq) / a;
  if (root < t_min || t_max < root) {
    root = (-half_b + sq) / a;
    if (root < t_min || t_max < root) return 0;
  }
  rec->t = root;
  rec->p = SFX(v3_add)(o, SFX(v3_mul)(d, root)); /* ray::at, ray.hpp:16-19 */
  V3 outward = SFX(v3_div)(SFX(v3_sub)(rec->p, c), radius);
  rec->front_face = SFX(v3_dot)(d, outward) < 0;
  rec->normal = rec->front_face ? outward : SFX(v3_neg)(outward);
  return 1;
}

/* hittable_list::hit_impl, hittable_list.hpp:32-58: ordered scan, shrinking closest_so_far,
 * the last accepted object (= closest, ties to the later index) wins. */
static int SFX(world_hit)(world_t* w, V3 o, V3 d, R t_min, R t_max, HIT* out) {
  R closest = t_max;
  int any = 0;
  HIT tmp;
  for (uint32_t i = 0; i < w->n; ++i) {
    w->tests++;
    if (SFX(sphere_hit)(&w->s[i], o, d, t_min, closest, &tmp)) {
      closest = tmp.t;
      tmp.id = i;
      *out = tmp;
      any = 1;
    }
  }
  return any;
}

/* Schlick, RTIOW (extension) — (1-c)^5 as an explicit left-to-right product */
static R SFX(reflectance)(R cosine, R ref_idx) {
  R r0 = ((R)1 - ref_idx) / ((R)1 + ref_idx);
  r0 = r0 * r0;
  R x = (R)1 - cosine;
  return r0 + ((R)1 - r0) * ((((x * x) * x) * x) * x);
}

/* scatter dispatch hittable_list.hpp:60-73 → sphere.hpp:50-54 → material.hpp */
static int SFX(scatter)(const yk_sphere* sp, V3 rd, const HIT* rec, mt_t* g, c3* att, V3* dir) {
  switch (sp->material) {
    case YK_MATERIAL_LAMBERTIAN: { /* material.hpp:50-59, random_unit_vector :33-36 */
      V3 ru = SFX(v3_random)(g, -1, 1);
      ru = SFX(v3_div)(ru, SFX(nsqrt)(SFX(v3_len2)(ru))); /* normalize(): *this /= length() */
      V3 sd = SFX(v3_add)(rec->normal, ru);
      if (SFX(v3_near_zero)(sd)) sd = rec->normal;
      *dir = sd;
      att->r = sp->albedo[0]; att->g = sp->albedo[1]; att->b = sp->albedo[2];
      return 1;
    }
    case YK_MATERIAL_METAL: { /* material.hpp:67-75 (+ fuzz extension) */
      V3 refl = SFX(v3_reflect)(SFX(v3_normalized)(rd), rec->normal);
      if (sp->fuzz > 0) { /* extension: + fuzz * random_in_unit_sphere (material.hpp:27-30) */
        /* the reference's random_in_unit_sphere returns random(-1,1).normalize() * uniform(0.01,
         * 0.99); g++ (its compiler, Makefile:1) evaluates that product's operands right to left,
         * so the length factor is drawn BEFORE the vector (pinned by the harness goldens) */
        R k = SFX(uniform)(g, (R)0.01, (R)0.99);
        V3 ru = SFX(v3_random)(g, -1, 1);
        ru = SFX(v3_div)(ru, SFX(nsqrt)(SFX(v3_len2)(ru)));
        refl = SFX(v3_add)(refl, SFX(v3_mul)(SFX(v3_mul)(ru, k), (R)sp->fuzz));
      }
      if (SFX(v3_dot)(refl, rec->normal) > 0) {
        *dir = refl;
        att->r = sp->albedo[0]; att->g = sp->albedo[1]; att->b = sp->albedo[2];
        return 1;
      }
      return 0;
    }
    case YK_MATERIAL_DIELECTRIC: { /* extension (RTIOW dielectric, yk-style arithmetic) */
      R ior = (R)sp->ior;
      R ratio = rec->front_face ? ((R)1 / ior) : ior;
      V3 unit = SFX(v3_normalized)(rd);
      R ct = SFX(v3_dot)(SFX(v3_neg)(unit), rec->normal);
      if (!(ct < (R)1)) ct = (R)1;
      R st = SFX(nsqrt)((R)1 - ct * ct);
      int cannot = ratio * st > (R)1;
      if (cannot || SFX(reflectance)(ct, ratio) > SFX(uniform)(g, 0, 1)) {
        *dir = SFX(v3_reflect)(unit, rec->normal);
      } else {
        V3 perp = SFX(v3_mul)(SFX(v3_add)(unit, SFX(v3_mul)(rec->normal, ct)), ratio);
        R pl = (R)1 - SFX(v3_len2)(perp);
        V3 par = SFX(v3_mul)(rec->normal, -SFX(nsqrt)(pl < 0 ? -pl : pl));
        *dir = SFX(v3_add)(perp, par);
      }
      att->r = 1.0; att->g = 1.0; att->b = 1.0;
      return 1;
    }
  }
  return 0;
}

/* raytracer<R, double>::ray_color, raytracer.hpp:19-37 — kept recursive, like the reference */
static c3 SFX(ray_color)(world_t* w, V3 o, V3 d, uint32_t depth, mt_t* g, uint64_t* segs) {
  c3 black = {0, 0, 0};
  if (depth == 0) return black;
  HIT rec;
  if (segs) (*segs)++;
  /* world.hit(r, 0.001, infinity<T>): the literal is converted to T (hittable.hpp:32) */
  if (SFX(world_hit)(w, o, d, (R)w->p->t_min, (R)INFINITY, &rec)) {
    c3 att;
    V3 nd;
    if (SFX(scatter)(&w->s[rec.id], d, &rec, g, &att, &nd)) {
      c3 in = SFX(ray_color)(w, rec.p, nd, depth - 1, g, segs);
      c3 r = {att.r * in.r, att.g * in.g, att.b * in.b};
      return r;
    }
    return black;
  }
  /* normalized(dir).y is an R; + 1.0 and everything after are double operations */
  double t = (SFX(v3_normalized)(d).y + 1.0) / 2;
  c3 r = {(1.0 - t) * 1.0 + t * 0.5, (1.0 - t) * 1.0 + t * 0.7, (1.0 - t) * 1.0 + t * 1.0};
  return r;
}

/* One sample after seeding: jitter source.cpp:160-164 (uniform_real_distribution<T>), get_ray
 * camera.hpp:29-32 (camera<T>: the record's doubles rounded to R) or the thin-lens extension. */
static c3 SFX(trace_sample)(world_t* w, mt_t* g, uint32_t y, uint32_t x, uint64_t* segs) {
  const yk_render_params* p = w->p;
  const yk_camera* cam = w->cam;
  R u = (x + SFX(uniform)(g, 0, 1)) / p->image_width;
  R v = (p->image_height - y - 1 + SFX(uniform)(g, 0, 1)) / p->image_height;
  V3 org = SFX(v3_of)(cam->origin);
  V3 dir = SFX(v3_add)(SFX(v3_add)(SFX(v3_of)(cam->lower_left_corner), SFX(v3_mul)(SFX(v3_of)(cam->horizontal), u)),
                       SFX(v3_mul)(SFX(v3_of)(cam->vertical), v));
  dir = SFX(v3_sub)(dir, org);
  if (cam->lens_radius > 0) { /* extension: random_in_unit_disk by rejection */
    R px, py;
    for (;;) {
      px = SFX(uniform)(g, -1, 1);
      py = SFX(uniform)(g, -1, 1);
      if (px * px + py * py < (R)1) break;
    }
    R lr = (R)cam->lens_radius;
    R rx = px * lr, ry = py * lr;
    V3 off = SFX(v3_add)(SFX(v3_mul)(SFX(v3_of)(cam->lens_u), rx), SFX(v3_mul)(SFX(v3_of)(cam->lens_v), ry));
    org = SFX(v3_add)(org, off);
    dir = SFX(v3_sub)(dir, off);
  }
  return SFX(ray_color)(w, org, dir, p->max_depth, g, segs);
}

#undef V3
#undef HIT
