// yk/ykgpu_bridge.hpp — the host-side adapter between a yk scene and the C-ABI (ykgpu.h).
//
// Flattens a world into yk_sphere records in tuple order (the order defines rec.id, the
// closest-hit tie-break and the scatter dispatch: /root/reference/yk/hittable_list.hpp:32-73)
// with std::apply over hittable_list::objects, and copies camera<T>'s public members
// (camera.hpp:34-37).  Only the public data members the reference's own types expose are
// read, so the same template compiles against either
//   * include/yk/scene.hpp (this repository's scene API), or
//   * the reference's yk/hittable_list.hpp + yk/sphere.hpp + yk/material.hpp + yk/camera.hpp
// — i.e. the reference's source.cpp can hand its world to the GPU unchanged.
//
// Then ykgpu::renderer runs the render loop of source.cpp:122-172 on the device — or on several:
// a device list (ykgpu_group_*, include/ykgpu.h; from the environment with devices_from_env())
// deals the image's rows over them — and returns the image_t bytes (source.cpp:70-71:
// row-major, row 0 at the top, RGB interleaved).
#pragma once

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <iomanip>
#include <ostream>
#include <stdexcept>
#include <initializer_list>
#include <string>
#include <tuple>
#include <type_traits>
#include <vector>

#include "../ykgpu.h"

namespace ykgpu {

namespace detail {
template <class M>
concept has_fuzz = requires(const M& m) { m.fuzz; };
template <class M>
concept has_ior = requires(const M& m) { m.ior; };
template <class W>
concept tuple_world = requires(const W& w) { std::tuple_size<std::decay_t<decltype(w.objects)>>::value; };
template <class C>
concept thin_lens = requires(const C& c) { c.lens_radius; c.lens_u; c.lens_v; };

template <class V>
void put3(double* dst, const V& v) {
  dst[0] = static_cast<double>(v.x);
  dst[1] = static_cast<double>(v.y);
  dst[2] = static_cast<double>(v.z);
}
template <class C>
void put_rgb(double* dst, const C& c) {
  dst[0] = static_cast<double>(c.r);
  dst[1] = static_cast<double>(c.g);
  dst[2] = static_cast<double>(c.b);
}
}  // namespace detail

// material.hpp:37-53 (lambertian) — the reference's and ours.
template <class U>
void set_material(yk_sphere& r, const yk::lambertian<U>& m) {
  r.material = YK_MATERIAL_LAMBERTIAN;
  detail::put_rgb(r.albedo, m.albedo);
}
// material.hpp:55-69 (metal); fuzz only exists in the extension.
template <class U>
void set_material(yk_sphere& r, const yk::metal<U>& m) {
  r.material = YK_MATERIAL_METAL;
  detail::put_rgb(r.albedo, m.albedo);
  if constexpr (detail::has_fuzz<yk::metal<U>>) r.fuzz = static_cast<double>(m.fuzz);
}
#ifdef YK_SCENE_HAS_EXTENSIONS
template <class U>
void set_material(yk_sphere& r, const yk::dielectric<U>& m) {
  r.material = YK_MATERIAL_DIELECTRIC;
  r.albedo[0] = r.albedo[1] = r.albedo[2] = 1.0;
  r.ior = static_cast<double>(m.ior);
}
#endif

// sphere.hpp:16-23
template <class S>
yk_sphere to_record(const S& s) {
  yk_sphere r;
  std::memset(&r, 0, sizeof r);
  detail::put3(r.center, s.center);
  r.radius = static_cast<double>(s.radius);
  set_material(r, s.material);
  return r;
}

// hittable_list<T, Hs...>: tuple order
template <class World>
  requires detail::tuple_world<World>
std::vector<yk_sphere> flatten(const World& w) {
  std::vector<yk_sphere> out;
  std::apply([&](const auto&... s) { (out.push_back(to_record(s)), ...); }, w.objects);
  return out;
}

#ifdef YK_SCENE_HAS_EXTENSIONS
// sphere_list<T>: insertion order
template <class T>
std::vector<yk_sphere> flatten(const yk::sphere_list<T>& w) {
  std::vector<yk_sphere> out;
  out.reserve(w.objects.size());
  for (const auto& e : w.objects) {
    yk_sphere r;
    std::memset(&r, 0, sizeof r);
    detail::put3(r.center, e.center);
    r.radius = static_cast<double>(e.radius);
    detail::put_rgb(r.albedo, e.albedo);
    r.fuzz = static_cast<double>(e.fuzz);
    r.ior = static_cast<double>(e.ior);
    using K = typename yk::sphere_list<T>::kind;
    r.material = e.k == K::lambertian ? YK_MATERIAL_LAMBERTIAN
                 : e.k == K::metal    ? YK_MATERIAL_METAL
                                      : YK_MATERIAL_DIELECTRIC;
    out.push_back(r);
  }
  return out;
}
#endif

// camera.hpp:34-37 (+ the thin-lens extension when present)
template <class Cam>
yk_camera camera_record(const Cam& c) {
  yk_camera r;
  std::memset(&r, 0, sizeof r);
  detail::put3(r.origin, c.origin);
  detail::put3(r.lower_left_corner, c.lower_left_corner);
  detail::put3(r.horizontal, c.horizontal);
  detail::put3(r.vertical, c.vertical);
  if constexpr (detail::thin_lens<Cam>) {
    detail::put3(r.lens_u, c.lens_u);
    detail::put3(r.lens_v, c.lens_v);
    r.lens_radius = static_cast<double>(c.lens_radius);
  }
  return r;
}

struct error : std::runtime_error {
  int code;
  error(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

inline void check(int rc, const char* where) {
  if (rc != YK_OK) throw error(rc, std::string(where) + ": " + ykgpu_last_error());
}

// The non-default yk_render_params modes (include/ykgpu.h).
struct render_options {
  uint32_t precision = YK_PRECISION_FP64;  // YK_PRECISION_FP32: render<float>
  uint32_t rng = YK_RNG_MT19937;           // YK_RNG_XOR128: yk::xor128 as the per-sample engine
  uint32_t seed_mode = YK_SEED_COUNTER;    // YK_SEED_RANDOM_DEVICE: the runtime build's seeding
  uint64_t seed_key = 0;                   // RANDOM_DEVICE key (0: a fresh one per call)
  double t_min = 0.001;                    // raytracer.hpp:27
};

// The devices a drop-in render uses, from the environment: YKGPU_DEVICES unset or empty → {0};
// "all" → every device of the node (ykgpu_device_count); otherwise a comma-separated list of
// device indices, repeats allowed ("0,1,2,3,4,5,6,7"; "0,0,0" runs three contexts on device 0).
inline std::vector<int> devices_from_env(const char* var = "YKGPU_DEVICES") {
  const char* e = std::getenv(var);
  std::vector<int> d;
  if (!e || !*e) return {0};
  const std::string v = e;
  if (v == "all") {
    int n = 0;
    check(ykgpu_device_count(&n), "ykgpu_device_count");
    for (int k = 0; k < n; ++k) d.push_back(k);
    if (d.empty()) throw error(YK_ERR_DEVICE, "YKGPU_DEVICES=all: no device");
    return d;
  }
  size_t i = 0;
  while (i < v.size()) {
    size_t used = 0;
    int k = 0;
    try {
      k = std::stoi(v.substr(i), &used);
    } catch (const std::exception&) {
      used = 0;
    }
    if (used == 0 || k < 0) throw error(YK_ERR_INVALID, std::string(var) + ": not a device list: " + v);
    d.push_back(k);
    i += used;
    if (i < v.size() && v[i] != ',') throw error(YK_ERR_INVALID, std::string(var) + ": not a device list: " + v);
    if (i < v.size()) {
      ++i;
      if (i == v.size()) throw error(YK_ERR_INVALID, std::string(var) + ": trailing ',' in " + v);
    }
  }
  if (d.empty()) throw error(YK_ERR_INVALID, std::string(var) + ": empty device list");
  // every index must name a device of this node (before any context is created)
  int n = 0;
  check(ykgpu_device_count(&n), (std::string(var) + ": ykgpu_device_count").c_str());
  for (int k : d)
    if (k >= n)
      throw error(YK_ERR_INVALID, std::string(var) + ": device " + std::to_string(k) + " of " + v + " does not exist (" +
                                      std::to_string(n) + " devices)");
  return d;
}

// The drop-in's render modes from the environment (all optional; unset = render() as the
// constexpr build computes it):
//   YKGPU_SEED      "counter" (seed0 + (y*W + x)*spp + s, source.cpp:154-158) or "random_device"
//                   (the runtime build's per-sample std::random_device seeding, source.cpp:159:
//                   a fresh key per call, not reproducible)
//   YKGPU_PRECISION "fp64" or "fp32" (render<float>, source.cpp:98-99)
//   YKGPU_RNG       "mt19937" or "xor128" (yk::xor128 as the per-sample engine)
inline render_options options_from_env() {
  render_options o;
  auto pick = [](const char* var, std::initializer_list<std::pair<const char*, uint32_t>> names,
                 uint32_t dflt) -> uint32_t {
    const char* e = std::getenv(var);
    if (!e || !*e) return dflt;
    std::string all;
    for (const auto& n : names) {
      if (std::string(e) == n.first) return n.second;
      all += std::string(all.empty() ? "" : ", ") + n.first;
    }
    throw error(YK_ERR_INVALID, std::string(var) + ": " + e + " is not one of " + all);
  };
  o.seed_mode = pick("YKGPU_SEED", {{"counter", YK_SEED_COUNTER}, {"random_device", YK_SEED_RANDOM_DEVICE}}, o.seed_mode);
  o.precision = pick("YKGPU_PRECISION", {{"fp64", YK_PRECISION_FP64}, {"fp32", YK_PRECISION_FP32}}, o.precision);
  o.rng = pick("YKGPU_RNG", {{"mt19937", YK_RNG_MT19937}, {"xor128", YK_RNG_XOR128}}, o.rng);
  return o;
}

// The render loop of source.cpp:122-172 on the GPU: one device context, or — given several
// devices — a group of contexts over which the image's rows are dealt (tile row t → entry t mod k).
// Tracing (-l 3) always runs on one context of the first device.
class renderer {
 public:
  explicit renderer(int device = 0) : devices_{device} { check(ykgpu_context_create(device, &ctx_), "ykgpu_context_create"); }
  explicit renderer(const std::vector<int>& devices) : devices_(devices) {
    if (devices_.empty()) throw error(YK_ERR_INVALID, "empty device list");
    if (devices_.size() == 1)
      check(ykgpu_context_create(devices_[0], &ctx_), "ykgpu_context_create");
    else
      check(ykgpu_group_create(devices_.data(), (uint32_t)devices_.size(), &group_), "ykgpu_group_create");
  }
  ~renderer() {
    ykgpu_group_destroy(group_);
    ykgpu_context_destroy(ctx_);
  }
  renderer(const renderer&) = delete;
  renderer& operator=(const renderer&) = delete;

  const std::vector<int>& devices() const { return devices_; }

  template <class World, class Cam>
  void set_scene(const World& world, const Cam& cam) {
    set_records(flatten(world), camera_record(cam));
  }

  // already-flattened records (e.g. yk_scene_build output)
  void set_records(const std::vector<yk_sphere>& s, const yk_camera& c) {
    if (group_)
      check(ykgpu_group_set_scene(group_, s.data(), (uint32_t)s.size(), &c), "ykgpu_group_set_scene");
    else
      check(ykgpu_set_scene(ctx_, s.data(), (uint32_t)s.size(), &c), "ykgpu_set_scene");
    spheres_ = s;
    cam_ = c;
    ctx_scene_ = !group_;
  }

  // image_t bytes of the whole image: W*H*3, row 0 at the top (source.cpp:70-71,224-226)
  std::vector<uint8_t> render(uint32_t width, uint32_t height, uint32_t spp, uint32_t max_depth,
                              uint32_t seed0, double t_min = 0.001) {
    render_options o;
    o.t_min = t_min;
    return render(width, height, spp, max_depth, seed0, o);
  }

  std::vector<uint8_t> render(uint32_t width, uint32_t height, uint32_t spp, uint32_t max_depth,
                              uint32_t seed0, const render_options& o) {
    std::vector<uint8_t> img((size_t)width * height * 3);
    render_into(img.data(), width, height, spp, max_depth, seed0, o);
    return img;
  }

  // The same into the caller's W*H*3 bytes (the patched source.cpp's image_t, filled in place)
  void render_into(uint8_t* rgb, uint32_t width, uint32_t height, uint32_t spp, uint32_t max_depth,
                   uint32_t seed0, const render_options& o = render_options{}) {
    const yk_render_params p = params(width, height, spp, max_depth, seed0, o);
    if (group_)
      check(ykgpu_group_render(group_, &p, rgb), "ykgpu_group_render");
    else
      check(ykgpu_render(ctx_, &p, rgb), "ykgpu_render");
  }

  static yk_render_params params(uint32_t width, uint32_t height, uint32_t spp, uint32_t max_depth,
                                 uint32_t seed0, const render_options& o) {
    yk_render_params p;
    std::memset(&p, 0, sizeof p);
    p.image_width = width;
    p.image_height = height;
    p.samples_per_pixel = spp;
    p.max_depth = max_depth;
    p.seed0 = seed0;
    p.row_begin = 0;
    p.row_count = height;
    p.row_stride = 1;
    p.precision = o.precision;
    p.rng = o.rng;
    p.seed_mode = o.seed_mode;
    p.seed_key = o.seed_key;
    p.t_min = o.t_min;
    return p;
  }

  // ray_color's rays (verbose level 3) of every sample of `rows` image rows from row_begin:
  // rays[(i*max_rays + k)*6 + {0..5}] = origin xyz, direction xyz of call k of sample
  // i = (row*W + x)*spp + s; counts[i] = its number of ray_color calls (include/ykgpu.h)
  void trace(uint32_t width, uint32_t height, uint32_t spp, uint32_t max_depth, uint32_t seed0,
             uint32_t row_begin, uint32_t rows, uint32_t max_rays, std::vector<double>& rays,
             std::vector<uint32_t>& counts, const render_options& o = {}) {
    yk_render_params p = params(width, height, spp, max_depth, seed0, o);
    p.row_begin = row_begin;
    p.row_count = rows;
    const size_t n = (size_t)rows * width * spp;
    rays.assign(n * max_rays * 6, 0.0);
    counts.assign(n, 0);
    trace_context();
    check(ykgpu_render_trace(ctx_, &p, max_rays, rays.data(), counts.data()), "ykgpu_render_trace");
  }

  // The console output of render()'s loop for the image just rendered, in the reference's order:
  // "(row,col)" per pixel at verbose >= 1 (source.cpp:128-135), "(row,col,sam)" per sample at
  // verbose >= 2 (:140-152) and, at verbose > 2, each ray ray_color is called with
  // (raytracer.hpp:21-25), the ray at depth 0 included.  The reference prints them while it
  // renders; here they follow the device's render.
  void print_verbose(std::ostream& os, uint32_t width, uint32_t height, uint32_t spp, uint32_t max_depth,
                     uint32_t seed0, uint32_t verbose, const render_options& o = {}) {
    if (!verbose) return;
    const auto w = [](uint32_t n) { return (int)(std::ceil(std::log10(n)) - 1); };
    const uint32_t max_rays = max_depth + 1;
    // row bands of at most ~256 MB of rays
    const size_t per_row = (size_t)width * spp * max_rays * 6 * sizeof(double);
    const uint32_t band = verbose > 2 ? (uint32_t)std::max<size_t>(1, (256u << 20) / std::max<size_t>(1, per_row)) : height;
    std::vector<double> rays;
    std::vector<uint32_t> counts;
    for (uint32_t y0 = 0; y0 < height; y0 += band) {
      const uint32_t rows = std::min(band, height - y0);
      if (verbose > 2) trace(width, height, spp, max_depth, seed0, y0, rows, max_rays, rays, counts, o);
      for (uint32_t y = y0; y < y0 + rows; ++y)
        for (uint32_t x = 0; x < width; ++x) {
          os << "(row,col) : " << '(' << std::setw(w(height)) << y << ',' << std::setw(w(width)) << x << ')'
             << std::endl;
          if (verbose < 2) continue;
          for (uint32_t s = 0; s < spp; ++s) {
            os << "(row,col,sam) : " << '(' << std::setw(w(height)) << y << ',' << std::setw(w(width)) << x << ','
               << std::setw(w(spp)) << s << ')' << std::endl;
            if (verbose < 3) continue;
            const size_t i = ((size_t)(y - y0) * width + x) * spp + s;
            for (uint32_t k = 0; k < counts[i] && k < max_rays; ++k) {
              const double* r = &rays[(i * max_rays + k) * 6];
              os << "ray { origin : (" << r[0] << ", " << r[1] << ", " << r[2] << "), direction : (" << r[3]
                 << ", " << r[4] << ", " << r[5] << ") }" << '\n';
            }
          }
        }
    }
  }

  // the last render's statistics (a group: the whole call, include/ykgpu.h)
  yk_render_stats stats() {
    yk_render_stats s;
    if (group_)
      check(ykgpu_group_get_stats(group_, -1, &s), "ykgpu_group_get_stats");
    else
      check(ykgpu_get_stats(ctx_, &s), "ykgpu_get_stats");
    return s;
  }

 private:
  // a group traces on a context of its first device, created on first use with the scene
  void trace_context() {
    if (!ctx_) check(ykgpu_context_create(devices_[0], &ctx_), "ykgpu_context_create");
    if (!ctx_scene_) {
      check(ykgpu_set_scene(ctx_, spheres_.data(), (uint32_t)spheres_.size(), &cam_), "ykgpu_set_scene");
      ctx_scene_ = true;
    }
  }

  std::vector<int> devices_;
  ykgpu_context* ctx_ = nullptr;
  ykgpu_group* group_ = nullptr;
  std::vector<yk_sphere> spheres_;
  yk_camera cam_{};
  bool ctx_scene_ = false;
};

}  // namespace ykgpu
