// oracle/ref_harness.cpp — TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// A driver of our own that #includes the reference's headers IN PLACE (-I/root/reference,
// nothing copied) and runs the reference's per-pixel loop deterministically, so that golden
// fixtures can be generated from the reference itself.  It is compiled by oracle/Makefile into
// oracle/_ref/ (git-ignored) only when /root/reference exists.
//
// The loop below has the shape of /root/reference/source.cpp:122-172 with the seed that the
// reference's constexpr build uses (source.cpp:118-120,154-158):
//     mt19937 gen(seed0 + (y*W + x)*spp + s)     (uint32 arithmetic, wraps mod 2^32)
// instead of std::random_device (source.cpp:159), which is what makes the output reproducible.
// The per-pixel sum is the same std::transform_reduce over iota(0,spp) (source.cpp:137-167) and
// the quantisation is a call-for-call restatement of to_color3b (source.cpp:73-83) built from the
// reference's own color3 / math::sqrt.
//
// Scenes are compile-time hittable_list tuples made only of reference types (sphere, lambertian,
// metal; yk/sphere.hpp, yk/material.hpp):
//   ref4     — source.cpp:103-112 verbatim values (the reference's only scene)
//   lambert3 — the same spheres with every material lambertian (BASELINE config 1 wording)
//   mixed12  — 12 spheres incl. an exact duplicate (tie-break rule of hittable_list.hpp:32-58)
//   walls2   — two facing lambertian walls: long paths (RNG draws past 227 / 624)
//
// Modes:
//   ref_harness render  <scene> W H spp depth seed0 out.rgb [out.sums]
//   ref_harness samples <scene> W H spp depth seed0 y x s [y x s ...]   (per-sample colours, hex)
//   ref_harness kat                                                   (RNG / sqrt / canonical KATs)
//   render32 / samples32: the same with T = float (render<float>(); radius literals as T(...))
//   render_x128 / samples_x128 / render32_x128 / samples32_x128: the engine is the reference's
//     yk::xor128 (random.hpp:18-41) seeded with the same per-sample counter, in place of mt19937
//   verbose <scene> W H spp depth seed0 level: the loop's console output at that verbose level,
//     the rays printed by the reference's ray_color itself (the -l 3 fixture)
//   render_file / samples_file (and the 32 / _x128 forms): <scene> is a scene file of 5, 24 or 48
//     spheres (configs 2-5 content: dielectric, fuzzed metal, thin-lens camera; see below)
#include <algorithm>
#include <cmath>
#include <iomanip>
#include <iostream>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <limits>
#include <numeric>
#include <ranges>
#include <string>
#include <vector>

#include "yk/camera.hpp"
#include "yk/color.hpp"
#include "yk/config.hpp"
#include "yk/hittable.hpp"
#include "yk/hittable_list.hpp"
#include "yk/material.hpp"
#include "yk/math.hpp"
#include "yk/random.hpp"
#include "yk/ray.hpp"
#include "yk/raytracer.hpp"
#include "yk/sphere.hpp"
#include "yk/vec3.hpp"

namespace {

template <class T>
using P = yk::pos3<T, yk::world_tag>;
using L = yk::lambertian<double>;
using M = yk::metal<double>;

// Counts u32 draws so fixtures can record stream consumption (values are untouched).
template <class E>
struct counting_gen {
  E* g;
  std::uint64_t n = 0;
  using result_type = typename E::result_type;
  static constexpr result_type min() { return E::min(); }
  static constexpr result_type max() { return E::max(); }
  result_type operator()() { ++n; return (*g)(); }
};

template <class T>
auto scene_ref4() {
  return yk::hittable_list<T>{}
      .add(yk::sphere(P<T>(0, 0, -1), T(0.5), L({0.7, 0.3, 0.3})))
      .add(yk::sphere(P<T>(0, -100.5, -1), T(100.0), L({0.8, 0.8, 0.0})))
      .add(yk::sphere(P<T>(-1.0, 0.0, -1.0), T(0.5), M({0.8, 0.8, 0.8})))
      .add(yk::sphere(P<T>(1.0, 0.0, -1.0), T(0.5), M({0.8, 0.6, 0.2})));
}

template <class T>
auto scene_lambert3() {
  return yk::hittable_list<T>{}
      .add(yk::sphere(P<T>(0, 0, -1), T(0.5), L({0.7, 0.3, 0.3})))
      .add(yk::sphere(P<T>(0, -100.5, -1), T(100.0), L({0.8, 0.8, 0.0})))
      .add(yk::sphere(P<T>(-1.0, 0.0, -1.0), T(0.5), L({0.8, 0.8, 0.8})));
}

template <class T>
auto scene_mixed12() {
  return yk::hittable_list<T>{}
      .add(yk::sphere(P<T>(0, -100.5, -1), T(100.0), L({0.8, 0.8, 0.0})))
      .add(yk::sphere(P<T>(0, 0, -1), T(0.5), L({0.1, 0.2, 0.5})))
      .add(yk::sphere(P<T>(-1.0, 0.0, -1.0), T(0.5), M({0.8, 0.8, 0.8})))
      .add(yk::sphere(P<T>(1.0, 0.0, -1.0), T(0.5), M({0.8, 0.6, 0.2})))
      .add(yk::sphere(P<T>(0, 0, -1), T(0.5), M({0.9, 0.9, 0.9})))
      .add(yk::sphere(P<T>(-0.5, 0.6, -1.5), T(0.3), L({0.9, 0.1, 0.1})))
      .add(yk::sphere(P<T>(0.5, 0.6, -1.5), T(0.3), M({0.2, 0.9, 0.2})))
      .add(yk::sphere(P<T>(0, -0.3, -0.6), T(0.15), L({0.2, 0.2, 0.9})))
      .add(yk::sphere(P<T>(0.3, 0.1, -0.45), T(0.1), M({0.95, 0.95, 0.95})))
      .add(yk::sphere(P<T>(-0.35, -0.35, -0.7), T(0.12), L({0.5, 0.9, 0.5})))
      .add(yk::sphere(P<T>(0, 1.2, -2.5), T(0.6), L({0.7, 0.7, 0.7})))
      .add(yk::sphere(P<T>(1.0, 0.0, -1.0), T(0.25), L({0.3, 0.3, 0.3})));
}

// two huge facing lambertian walls: long bounce chains (draws > 227 and > 624 at depth 200)
template <class T>
auto scene_walls2() {
  return yk::hittable_list<T>{}
      .add(yk::sphere(P<T>(0, -300.5, -1), T(300.0), L({0.9, 0.85, 0.8})))
      .add(yk::sphere(P<T>(0, 300.5, -1), T(300.0), L({0.8, 0.9, 0.95})));
}

struct job {
  std::uint32_t W, H, spp, depth, seed0;
};

// ---- BASELINE configs 2-5 content through the reference's own integrator ---------------------
// The reference has no dielectric, no fuzzed metal and no positionable camera, but
// its integrator takes any material type: concepts::material is `true` (material.hpp:22-23),
// hittable_list::scatter dispatches by rec.id (hittable_list.hpp:60-73) to sphere::scatter_impl
// (sphere.hpp:50-54), which calls the material, and ray_color multiplies and recurses
// (raytracer.hpp:19-37).  The three extension bodies below are OURS — they restate
// oracle/yk_oracle_path.h and the kernel — and everything around them is the reference's code:
// ray_color, the ordered closest-hit fold, sphere::hit_impl, set_face_normal, mt19937,
// uniform_real_distribution, math::sqrt, reflect, normalized and random_in_unit_sphere.  A golden
// rendered here therefore pins the extensions' RNG interleaving and their integration to the
// reference; only the scatter bodies and the camera's lens remain unpinned.

// fuzzed metal: metal::scatter (material.hpp:67-75) with RTIOW's `reflected + fuzz *
// random_in_unit_sphere()` — the reference's own random_in_unit_sphere (material.hpp:27-30), whose
// two operands g++ (the reference's compiler, Makefile:1) evaluates right to left: the length
// factor uniform(0.01, 0.99) is drawn BEFORE the vector.
template <class U>
struct fuzzy_metal {
  yk::color3<U> albedo;
  double fuzz;
  template <class T, class Gen>
  constexpr std::optional<std::pair<yk::color3<U>, yk::ray<T>>> scatter(const yk::ray<T>& r_in,
                                                                        const yk::hit_record<T>& rec,
                                                                        Gen& gen) const {
    auto reflected = reflect(r_in.direction.normalized(), rec.normal);
    reflected = reflected + T(fuzz) * yk::random_in_unit_sphere<T>(gen);
    auto scattered = yk::ray(rec.p, reflected);
    if (dot(scattered.direction, rec.normal) > 0) return std::make_pair(albedo, scattered);
    return std::nullopt;
  }
};

// dielectric (RTIOW): Snell with total internal reflection, Schlick's reflectance, attenuation 1
template <class U>
struct dielectric_ext {
  double ior;
  template <class T>
  static constexpr T reflectance(T cosine, T ref_idx) {
    T r0 = (T(1) - ref_idx) / (T(1) + ref_idx);
    r0 = r0 * r0;
    T x = T(1) - cosine;
    return r0 + (T(1) - r0) * ((((x * x) * x) * x) * x);
  }
  template <class T, class Gen>
  constexpr std::optional<std::pair<yk::color3<U>, yk::ray<T>>> scatter(const yk::ray<T>& r_in,
                                                                        const yk::hit_record<T>& rec,
                                                                        Gen& gen) const {
    const T ir = T(ior);
    const T ratio = rec.front_face ? (T(1) / ir) : ir;
    const auto unit = r_in.direction.normalized();
    T ct = dot(-unit, rec.normal);
    if (!(ct < T(1))) ct = T(1);
    const T st = yk::math::sqrt(T(1) - ct * ct);
    const bool cannot = ratio * st > T(1);
    yk::vec3<T> dir;
    if (cannot || reflectance(ct, ratio) > yk::uniform_real_distribution<T>(0, 1)(gen)) {
      dir = reflect(unit, rec.normal);
    } else {
      const auto perp = (unit + ct * rec.normal) * ratio;
      const T pl = T(1) - perp.length_squared();
      dir = perp + rec.normal * (-yk::math::sqrt(pl < 0 ? -pl : pl));
    }
    return std::make_pair(yk::color3<U>(1.0, 1.0, 1.0), yk::ray(rec.p, dir));
  }
};

// one material type for every sphere of a scene file: dispatches to the reference's lambertian
// and metal (fuzz 0) or to the extensions above
struct any_material {
  std::uint32_t kind;  // 0 lambertian, 1 metal, 2 dielectric (include/ykgpu.h YK_MATERIAL_*)
  yk::color3<double> albedo;
  double fuzz, ior;
  template <class T, class Gen>
  constexpr std::optional<std::pair<yk::color3<double>, yk::ray<T>>> scatter(const yk::ray<T>& r,
                                                                             const yk::hit_record<T>& rec,
                                                                             Gen& gen) const {
    if (kind == 0) return yk::lambertian<double>(albedo).scatter(r, rec, gen);
    if (kind == 1) {
      if (fuzz > 0) return fuzzy_metal<double>{albedo, fuzz}.scatter(r, rec, gen);
      return yk::metal<double>(albedo).scatter(r, rec, gen);
    }
    return dielectric_ext<double>{ior}.scatter(r, rec, gen);
  }
};

// positionable thin-lens camera (RTIOW): the reference camera's get_ray (camera.hpp:29-32) as
// llc + u*horizontal + v*vertical - origin, the origin moved by a point of the lens disk drawn by
// rejection (x, then y, each uniform(-1, 1))
template <class T>
struct lens_camera {
  yk::vec3<T> origin, lower_left_corner, horizontal, vertical, lens_u, lens_v;
  T lens_radius;
  template <class Gen>
  constexpr yk::ray<T> get_ray(T u, T v, Gen& gen) const {
    auto org = origin;
    auto dir = lower_left_corner + u * horizontal + v * vertical - origin;
    if (lens_radius > 0) {
      T px, py;
      for (;;) {
        px = yk::uniform_real_distribution<T>(-1, 1)(gen);
        py = yk::uniform_real_distribution<T>(-1, 1)(gen);
        if (px * px + py * py < T(1)) break;
      }
      const T rx = px * lens_radius, ry = py * lens_radius;
      const auto off = lens_u * rx + lens_v * ry;
      org = org + off;
      dir = dir - off;
    }
    return yk::ray<T>{P<T>(org.x, org.y, org.z), dir};
  }
};

// scene files (include/ykgpu.h yk_scene_write: "yk-scene 1", one camera line, sphere lines)
struct file_sphere {
  double c[3], r, albedo[3], fuzz, ior;
  std::uint32_t kind;
};
struct scene_file {
  double cam[19];
  std::vector<file_sphere> s;
};
bool read_scene_file(const char* path, scene_file& out) {
  FILE* f = std::fopen(path, "r");
  if (!f) return false;
  char line[2048];
  bool cam = false;
  while (std::fgets(line, sizeof line, f)) {
    if (!std::strncmp(line, "camera", 6)) {
      const char* p = line + 6;
      for (int k = 0; k < 19; ++k) {
        char* e = nullptr;
        out.cam[k] = std::strtod(p, &e);
        p = e;
      }
      cam = true;
    } else if (!std::strncmp(line, "sphere", 6)) {
      file_sphere s{};
      char kind[32] = {0};
      if (std::sscanf(line + 6, "%31s %lf %lf %lf %lf %lf %lf %lf %lf %lf", kind, &s.c[0], &s.c[1], &s.c[2], &s.r,
                      &s.albedo[0], &s.albedo[1], &s.albedo[2], &s.fuzz, &s.ior) != 10)
        return false;
      s.kind = !std::strcmp(kind, "lambertian") ? 0u : !std::strcmp(kind, "metal") ? 1u : 2u;
      out.s.push_back(s);
    }
  }
  std::fclose(f);
  return cam;
}
template <class T>
lens_camera<T> file_camera(const scene_file& sf) {
  auto v = [&](int k) { return yk::vec3<T>{T(sf.cam[k]), T(sf.cam[k + 1]), T(sf.cam[k + 2])}; };
  return {v(0), v(3), v(6), v(9), v(12), v(15), T(sf.cam[18])};
}
template <class T, std::size_t I>
using file_sphere_t = yk::sphere<T, any_material>;
template <class T>
file_sphere_t<T, 0> make_sphere(const file_sphere& s) {
  return yk::sphere(P<T>(s.c[0], s.c[1], s.c[2]), T(s.r),
                    any_material{s.kind, {s.albedo[0], s.albedo[1], s.albedo[2]}, s.fuzz, s.ior});
}
// a compile-time tuple of N spheres filled from the file (the tuple API needs N at compile time)
template <class T, std::size_t... I>
auto file_world(const scene_file& sf, std::index_sequence<I...>) {
  return yk::hittable_list<T, file_sphere_t<T, I>...>(std::tuple<file_sphere_t<T, I>...>(make_sphere<T>(sf.s[I])...));
}

// T = double is render() as shipped (source.cpp:98); T = float is render<float>(): geometry,
// camera, canonicals (one draw each) and math::sqrt in float, colour still double
// (raytracer<T, double>, lambertian<double>).
// camera<T>::get_ray(u, v) (camera.hpp:29-32), or the lens camera's, which also draws
template <class T, class Cam, class Gen>
yk::ray<T> camera_ray(const Cam& cam, T u, T v, Gen& gen) {
  if constexpr (requires { cam.get_ray(u, v, gen); })
    return cam.get_ray(u, v, gen);
  else
    return cam.get_ray(u, v);
}

template <class T, class E, class World, class Cam>
yk::color3d sample_color(const World& world, const Cam& cam, const job& j, std::uint32_t y, std::uint32_t x,
                         std::uint32_t s, std::uint64_t* draws) {
  const yk::raytracer<T, double> tracer = {};
  E g(j.seed0 + (y * j.W + x) * j.spp + s);
  counting_gen<E> gen{&g};
  yk::uniform_real_distribution<T> dist(0, 1);
  T u = (x + dist(gen)) / j.W;
  T v = (j.H - y - 1 + dist(gen)) / j.H;
  auto c = tracer.ray_color(camera_ray<T>(cam, u, v, gen), world, j.depth, gen);
  if (draws) *draws = gen.n;
  return c;
}

template <class T, class E, class World, class Cam>
int render(const World& world, const Cam& cam, const job& j, const char* out_rgb, const char* out_sums) {
  std::vector<unsigned char> rgb(std::size_t(j.W) * j.H * 3);
  std::vector<double> sums(std::size_t(j.W) * j.H * 3);
  // YK_REF_ROWS="b:k" renders rows b, b + k, b + 2k, ... only (the others stay 0): k processes of
  // this loop then cover the image on k cores (bench.py reference_calibration; the reference's
  // own par mode, source.cpp:85-96, does not run)
  std::uint32_t y0 = 0, ystep = 1;
  if (const char* e = std::getenv("YK_REF_ROWS")) {
    char* rest = nullptr;
    y0 = std::strtoul(e, &rest, 10);
    if (rest && *rest == ':') ystep = std::max(1ul, std::strtoul(rest + 1, nullptr, 10));
  }
  for (std::uint32_t y = y0; y < j.H; y += ystep) {
    for (std::uint32_t x = 0; x < j.W; ++x) {
      auto iota = std::views::iota(0u, j.spp);
      yk::color3d pc = std::transform_reduce(
          iota.begin(), iota.end(), yk::color3d(0, 0, 0), std::plus{},
          [&](auto s) { return sample_color<T, E>(world, cam, j, y, x, s, nullptr); });
      const std::size_t i = std::size_t(y) * j.W + x;
      sums[3 * i + 0] = pc.r;
      sums[3 * i + 1] = pc.g;
      sums[3 * i + 2] = pc.b;
      // to_color3b, source.cpp:73-83
      auto [r, g, b] = pc / j.spp;
      yk::color3d c = {.r = yk::math::sqrt(r), .g = yk::math::sqrt(g), .b = yk::math::sqrt(b)};
      auto q = (c.clamped(0.0, 0.999) * 256).template to<std::uint8_t>();
      rgb[3 * i + 0] = q.r;
      rgb[3 * i + 1] = q.g;
      rgb[3 * i + 2] = q.b;
    }
  }
  FILE* f = std::fopen(out_rgb, "wb");
  if (!f) return 1;
  std::fwrite(rgb.data(), 1, rgb.size(), f);
  std::fclose(f);
  if (out_sums) {
    f = std::fopen(out_sums, "wb");
    if (!f) return 1;
    std::fwrite(sums.data(), sizeof(double), sums.size(), f);
    std::fclose(f);
  }
  return 0;
}

template <class T, class E, class World, class Cam>
int samples(const World& world, const Cam& cam, const job& j, int argc, char** argv) {
  std::printf("[\n");
  for (int k = 0; k + 2 < argc; k += 3) {
    std::uint32_t y = std::strtoul(argv[k], nullptr, 10);
    std::uint32_t x = std::strtoul(argv[k + 1], nullptr, 10);
    std::uint32_t s = std::strtoul(argv[k + 2], nullptr, 10);
    std::uint64_t n = 0;
    auto c = sample_color<T, E>(world, cam, j, y, x, s, &n);
    std::printf("  {\"y\": %u, \"x\": %u, \"s\": %u, \"draws\": %llu, \"rgb\": [\"%a\", \"%a\", \"%a\"]}%s\n",
                y, x, s, (unsigned long long)n, c.r, c.g, c.b, (k + 5 < argc) ? "," : "");
  }
  std::printf("]\n");
  return 0;
}

int kat() {
  std::printf("{\n  \"mt19937\": {\n");
  const std::uint32_t seeds[] = {5489u, 404u, 0u, 1u, 4294967295u, 123456789u};
  for (std::size_t k = 0; k < sizeof(seeds) / sizeof(seeds[0]); ++k) {
    yk::mt19937 g(seeds[k]);
    std::printf("    \"%u\": [", seeds[k]);
    // 1300 outputs: crosses the lazy-cursor limit (227), one full re-twist (624) and a second.
    for (int i = 0; i < 1300; ++i) std::printf("%s%llu", i ? ", " : "", (unsigned long long)g());
    std::printf("]%s\n", (k + 1 < sizeof(seeds) / sizeof(seeds[0])) ? "," : "");
  }
  std::printf("  },\n  \"canonical01\": {\n");
  for (std::size_t k = 0; k < sizeof(seeds) / sizeof(seeds[0]); ++k) {
    yk::mt19937 g(seeds[k]);
    yk::uniform_real_distribution<double> d01(0, 1), dpm(-1, 1);
    std::printf("    \"%u\": [", seeds[k]);
    for (int i = 0; i < 64; ++i) {
      double v = (i % 3 == 2) ? dpm(g) : d01(g);  // pattern 0,1 / -1,1 mixes both ranges
      std::printf("%s\"%a\"", i ? ", " : "", v);
    }
    std::printf("]%s\n", (k + 1 < sizeof(seeds) / sizeof(seeds[0])) ? "," : "");
  }
  std::printf("  },\n  \"canonical01_f32\": {\n");
  for (std::size_t k = 0; k < sizeof(seeds) / sizeof(seeds[0]); ++k) {
    yk::mt19937 g(seeds[k]);
    yk::uniform_real_distribution<float> d01(0, 1), dpm(-1, 1);
    std::printf("    \"%u\": [", seeds[k]);
    for (int i = 0; i < 64; ++i) {
      float v = (i % 3 == 2) ? dpm(g) : d01(g);
      std::printf("%s\"%a\"", i ? ", " : "", (double)v);
    }
    std::printf("]%s\n", (k + 1 < sizeof(seeds) / sizeof(seeds[0])) ? "," : "");
  }
  std::printf("  },\n  \"xor128\": {\n");
  for (std::size_t k = 0; k < sizeof(seeds) / sizeof(seeds[0]); ++k) {
    yk::xor128 g(seeds[k]);
    std::printf("    \"%u\": [", seeds[k]);
    for (int i = 0; i < 256; ++i) std::printf("%s%llu", i ? ", " : "", (unsigned long long)g());
    std::printf("]%s\n", (k + 1 < sizeof(seeds) / sizeof(seeds[0])) ? "," : "");
  }
  std::printf("  },\n  \"canonical01_x128\": {\n");
  for (std::size_t k = 0; k < sizeof(seeds) / sizeof(seeds[0]); ++k) {
    yk::xor128 g(seeds[k]);
    yk::uniform_real_distribution<double> d01(0, 1), dpm(-1, 1);
    std::printf("    \"%u\": [", seeds[k]);
    for (int i = 0; i < 64; ++i) {
      double v = (i % 3 == 2) ? dpm(g) : d01(g);
      std::printf("%s\"%a\"", i ? ", " : "", v);
    }
    std::printf("]%s\n", (k + 1 < sizeof(seeds) / sizeof(seeds[0])) ? "," : "");
  }
  std::printf("  },\n  \"newton_sqrt_f32\": [");
  {
    std::vector<float> fs = {0.0f, 1.0f, 2.0f, 4.0f, 0.25f, 1e-30f, 1e-45f, 1e30f, 3.0f, 0.999f, 1e-8f,
                             3.4e38f, 1.2e-38f};
    std::uint64_t sf = 0x2545F4914F6CDD1Dull;
    for (int i = 0; i < 500; ++i) {
      sf = sf * 6364136223846793005ull + 1442695040888963407ull;
      float m = 1.0f + float(sf >> 41) * 0x1p-23f;
      int e = int((sf >> 3) % 60) - 30;
      fs.push_back(std::ldexp(m, e));
    }
    for (std::size_t i = 0; i < fs.size(); ++i)
      std::printf("%s[\"%a\", \"%a\"]", i ? ", " : "", (double)fs[i], (double)yk::math::sqrt(fs[i]));
  }
  std::printf("],\n  \"newton_sqrt\": [");
  // deterministic spread of inputs (LCG-scrambled mantissas over many binades) plus edges
  std::vector<double> xs = {0.0, 1.0, 2.0, 4.0, 0.25, 1e-300, 5e-324, 1e300, 3.0, 0.999, 1e-8};
  std::uint64_t st = 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < 500; ++i) {
    st = st * 6364136223846793005ull + 1442695040888963407ull;
    double m = 1.0 + double(st >> 11) * 0x1p-53;
    int e = int((st >> 3) % 60) - 30;
    xs.push_back(std::ldexp(m, e));
  }
  for (std::size_t i = 0; i < xs.size(); ++i)
    std::printf("%s[\"%a\", \"%a\"]", i ? ", " : "", xs[i], yk::math::sqrt(xs[i]));
  std::printf("]\n}\n");
  return 0;
}

// The console output of source.cpp's loop at verbose level `lv` (source.cpp:128-152 restated,
// in its pixel / sample order) with the reference's own ray_color printing every ray it is called
// with at level 3 (raytracer.hpp:21-25): the fixture of the drop-in's `-l 3`.
template <class T, class E, class World, class Cam>
int verbose_lines(const World& world, const Cam& cam, const job& j, std::uint32_t lv) {
  std::ios::sync_with_stdio(false);
  yk::verbose = lv;
  const auto w = [](std::uint32_t n) { return (int)(std::ceil(std::log10(n)) - 1); };
  for (std::uint32_t y = 0; y < j.H; ++y)
    for (std::uint32_t x = 0; x < j.W; ++x) {
      std::cout << "(row,col) : " << '(' << std::setw(w(j.H)) << y << ',' << std::setw(w(j.W)) << x << ')'
                << std::endl;
      for (std::uint32_t s = 0; s < j.spp; ++s) {
        if (lv > 1)
          std::cout << "(row,col,sam) : " << '(' << std::setw(w(j.H)) << y << ',' << std::setw(w(j.W)) << x << ','
                    << std::setw(w(j.spp)) << s << ')' << std::endl;
        sample_color<T, E>(world, cam, j, y, x, s, nullptr);
      }
    }
  std::cout.flush();
  return 0;
}

template <class T, class E, class World, class Cam = yk::camera<T>>
int dispatch_world(const World& w, const char* mode, const job& j, int argc, char** argv, const Cam& cam = {}) {
  if (!std::strncmp(mode, "render", 6)) return render<T, E>(w, cam, j, argv[0], argc > 1 ? argv[1] : nullptr);
  if (!std::strncmp(mode, "verbose", 7)) return verbose_lines<T, E>(w, cam, j, argc > 0 ? std::atoi(argv[0]) : 3);
  return samples<T, E>(w, cam, j, argc, argv);
}

// a scene file (configs 2-5 content): N spheres in a compile-time tuple, the lens camera
template <class T, class E, std::size_t N>
int dispatch_file_n(const scene_file& sf, const char* mode, const job& j, int argc, char** argv) {
  return dispatch_world<T, E>(file_world<T>(sf, std::make_index_sequence<N>{}), mode, j, argc, argv,
                              file_camera<T>(sf));
}
template <class T, class E>
int dispatch_file(const std::string& path, const char* mode, const job& j, int argc, char** argv) {
  scene_file sf;
  if (!read_scene_file(path.c_str(), sf)) {
    std::fprintf(stderr, "cannot read scene file %s\n", path.c_str());
    return 2;
  }
  switch (sf.s.size()) {
    case 5: return dispatch_file_n<T, E, 5>(sf, mode, j, argc, argv);
    case 24: return dispatch_file_n<T, E, 24>(sf, mode, j, argc, argv);
    case 48: return dispatch_file_n<T, E, 48>(sf, mode, j, argc, argv);
  }
  std::fprintf(stderr, "scene files of 5, 24 or 48 spheres only (tuple sizes compiled in), got %zu\n", sf.s.size());
  return 2;
}

template <class T, class E>
int dispatch(const std::string& scene, const char* mode, const job& j, int argc, char** argv) {
  if (std::strstr(mode, "_file")) return dispatch_file<T, E>(scene, mode, j, argc, argv);
  if (scene == "ref4") return dispatch_world<T, E>(scene_ref4<T>(), mode, j, argc, argv);
  if (scene == "lambert3") return dispatch_world<T, E>(scene_lambert3<T>(), mode, j, argc, argv);
  if (scene == "mixed12") return dispatch_world<T, E>(scene_mixed12<T>(), mode, j, argc, argv);
  if (scene == "walls2") return dispatch_world<T, E>(scene_walls2<T>(), mode, j, argc, argv);
  std::fprintf(stderr, "unknown scene %s\n", scene.c_str());
  return 2;
}

}  // namespace

int main(int argc, char** argv) {
  if (argc >= 2 && !std::strcmp(argv[1], "kat")) return kat();
  if (argc < 9) {
    std::fprintf(stderr, "usage: %s render|samples scene W H spp depth seed0 ...\n", argv[0]);
    return 2;
  }
  job j{(std::uint32_t)std::strtoul(argv[3], nullptr, 10), (std::uint32_t)std::strtoul(argv[4], nullptr, 10),
        (std::uint32_t)std::strtoul(argv[5], nullptr, 10), (std::uint32_t)std::strtoul(argv[6], nullptr, 10),
        (std::uint32_t)std::strtoul(argv[7], nullptr, 10)};
  const std::string scene = argv[2];
  // render32 / samples32: the same loop instantiated with T = float; a "_x128" suffix seeds the
  // reference's other engine, yk::xor128 (random.hpp:18-41), instead of yk::mt19937
  const bool f32 = std::strstr(argv[1], "32") != nullptr;
  const bool x128 = std::strstr(argv[1], "_x128") != nullptr;
  if (x128)
    return f32 ? dispatch<float, yk::xor128>(scene, argv[1], j, argc - 8, argv + 8)
               : dispatch<double, yk::xor128>(scene, argv[1], j, argc - 8, argv + 8);
  return f32 ? dispatch<float, yk::mt19937>(scene, argv[1], j, argc - 8, argv + 8)
             : dispatch<double, yk::mt19937>(scene, argv[1], j, argc - 8, argv + 8);
}
