// yk/scene.hpp — host-side scene description API of the drop-in renderer.
//
// Source-compatible with the scene-building code of the reference's render()
// (/root/reference/source.cpp:100-112):
//
//   const auto world = yk::hittable_list<double>{}
//       .add(yk::sphere(yk::pos3<double, yk::world_tag>(0, 0, -1), 0.5,
//                       yk::lambertian<double>({0.7, 0.3, 0.3})))
//       .add(...);
//   const yk::camera<double> cam = {};
//
// The types keep the reference's public data members (vec3::x/y/z, color3::r/g/b,
// sphere::center/radius/material, lambertian/metal::albedo, camera::origin/
// lower_left_corner/horizontal/vertical, hittable_list::objects) because those are what the
// bridge (ykgpu_bridge.hpp) reads — so the bridge works on the reference's own types too.
// What is NOT here: the per-sample arithmetic (hit, scatter, ray_color); that runs on the GPU
// behind include/ykgpu.h.
//
// Extensions for BASELINE configs 2-5 (no reference code; parity unpinned): metal fuzz,
// dielectric, a positionable thin-lens camera, and sphere_list — a runtime-sized world for
// scenes the compile-time tuple cannot hold (~500 spheres).
#pragma once

#include <cmath>
#include <cstdint>
#include <tuple>
#include <type_traits>
#include <vector>

#define YK_SCENE_HAS_EXTENSIONS 1

namespace yk {

// ---- tags and vectors (reference: yk/vec3.hpp:13-27,205-209) ------------------------------
struct tag_base {};
struct default_tag : tag_base {};
struct world_tag : default_tag {};
struct camera_tag : world_tag {};

template <class T, class Tag = default_tag>
struct vec3 {
  T x, y, z;
};
template <class T, class Tag>
using pos3 = vec3<T, Tag>;
using vec3d = vec3<double>;

template <class T, class A, class B>
constexpr vec3<T, A> operator+(const vec3<T, A>& l, const vec3<T, B>& r) { return {l.x + r.x, l.y + r.y, l.z + r.z}; }
template <class T, class A, class B>
constexpr vec3<T, A> operator-(const vec3<T, A>& l, const vec3<T, B>& r) { return {l.x - r.x, l.y - r.y, l.z - r.z}; }
template <class T, class A>
constexpr vec3<T, A> operator*(const vec3<T, A>& v, T s) { return {v.x * s, v.y * s, v.z * s}; }
template <class T, class A>
constexpr vec3<T, A> operator/(const vec3<T, A>& v, T s) { return {v.x / s, v.y / s, v.z / s}; }

// ---- colours (reference: yk/color.hpp:13-24,119-120) ---------------------------------------
template <class T>
struct color3 {
  using value_type = T;
  T r, g, b;
};
using color3b = color3<uint8_t>;
using color3d = color3<double>;

// ---- materials (reference: yk/material.hpp:37-69) ------------------------------------------
template <class U>
struct lambertian {
  color3<U> albedo;
  constexpr lambertian(const color3<U>& a) : albedo(a) {}
};

template <class U>
struct metal {
  color3<U> albedo;
  U fuzz = 0;  // extension; 0 = the reference's mirror metal (no random draw)
  constexpr metal(const color3<U>& a, U f = 0) : albedo(a), fuzz(f) {}
};

template <class U>
struct dielectric {  // extension (RTIOW glass)
  U ior;
  constexpr explicit dielectric(U index_of_refraction) : ior(index_of_refraction) {}
};

// ---- sphere (reference: yk/sphere.hpp:16-23,58) -------------------------------------------
template <class T, class M>
struct sphere {
  pos3<T, world_tag> center;
  T radius;
  M material;
  constexpr sphere(pos3<T, world_tag> c, T r, M m) : center(c), radius(r), material(m) {}
};
template <class T, class M>
sphere(pos3<T, world_tag>, T, M) -> sphere<T, M>;

// ---- world: compile-time tuple (reference: yk/hittable_list.hpp:18-30) --------------------
template <class T, class... Hs>
struct hittable_list {
  std::tuple<Hs...> objects = {};
  constexpr hittable_list() = default;
  constexpr explicit hittable_list(std::tuple<Hs...> o) : objects(std::move(o)) {}
  template <class H>
  [[nodiscard]] constexpr hittable_list<T, Hs..., H> add(H h) const {
    return hittable_list<T, Hs..., H>(std::tuple_cat(objects, std::tuple<H>(std::move(h))));
  }
};

// ---- world: runtime list (extension) -----------------------------------------------------
template <class T>
struct sphere_list {
  enum class kind : uint8_t { lambertian, metal, dielectric };
  struct entry {
    pos3<T, world_tag> center;
    T radius;
    kind k;
    color3<T> albedo;
    T fuzz, ior;
  };
  std::vector<entry> objects;
  sphere_list& add(const sphere<T, lambertian<T>>& s) {
    objects.push_back({s.center, s.radius, kind::lambertian, s.material.albedo, 0, 0});
    return *this;
  }
  sphere_list& add(const sphere<T, metal<T>>& s) {
    objects.push_back({s.center, s.radius, kind::metal, s.material.albedo, s.material.fuzz, 0});
    return *this;
  }
  sphere_list& add(const sphere<T, dielectric<T>>& s) {
    objects.push_back({s.center, s.radius, kind::dielectric, {1, 1, 1}, 0, s.material.ior});
    return *this;
  }
};

// ---- camera (reference: yk/camera.hpp:14-38; same default construction) -------------------
template <class T>
struct camera {
  pos3<T, world_tag> origin;
  pos3<T, camera_tag> lower_left_corner;
  vec3<T> horizontal;
  vec3<T> vertical;
  // thin-lens extension (zero for the reference camera)
  vec3<T> lens_u{0, 0, 0}, lens_v{0, 0, 0};
  T lens_radius = 0;

  constexpr camera() {
    const T aspect_ratio = 16.0 / 9.0, viewport_height = 2.0;
    const T viewport_width = aspect_ratio * viewport_height, focal_length = 1.0;
    origin = {0, 0, 0};
    horizontal = {viewport_width, 0.0, 0.0};
    vertical = {0.0, viewport_height, 0.0};
    const pos3<T, camera_tag> o{0, 0, 0};
    lower_left_corner = o - horizontal / T(2) - vertical / T(2) - vec3<T>{0, 0, focal_length};
  }

  // positionable thin-lens camera (extension; RTIOW book 1 ch. 12-13)
  static camera look(pos3<T, world_tag> from, pos3<T, world_tag> at, vec3<T> vup, T vfov_deg,
                     T aspect, T aperture, T focus_dist) {
    auto dot = [](auto a, auto b) { return a.x * b.x + a.y * b.y + a.z * b.z; };
    auto unit = [&](auto a) { return a / std::sqrt(dot(a, a)); };
    auto cross = [](auto a, auto b) {
      return vec3<T>{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
    };
    const T h = std::tan(vfov_deg * T(M_PI) / T(180) / 2);
    const T vh = 2 * h, vw = aspect * vh;
    const vec3<T> w = unit(vec3<T>{from.x - at.x, from.y - at.y, from.z - at.z});
    const vec3<T> u = unit(cross(vup, w)), v = cross(w, u);
    camera c;
    c.origin = from;
    c.horizontal = u * (focus_dist * vw);
    c.vertical = v * (focus_dist * vh);
    const pos3<T, camera_tag> f{from.x, from.y, from.z};
    c.lower_left_corner = f - c.horizontal / T(2) - c.vertical / T(2) - w * focus_dist;
    c.lens_u = u;
    c.lens_v = v;
    c.lens_radius = aperture / 2;
    return c;
  }
};

}  // namespace yk
