// yk_host.cpp — host-side scene helpers of the C-ABI (no device code): the reference camera,
// the positionable camera extension and the named scenes of the BASELINE configs.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ykgpu.h"

namespace {

struct d3 {
  double x, y, z;
};
d3 operator-(d3 a, d3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
d3 operator*(d3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }
d3 operator/(d3 a, double s) { return {a.x / s, a.y / s, a.z / s}; }
double dot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
d3 cross(d3 a, d3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
d3 unit(d3 a) { return a / std::sqrt(dot(a, a)); }
void put(double* dst, d3 v) {
  dst[0] = v.x;
  dst[1] = v.y;
  dst[2] = v.z;
}

// Scene generator RNG: mt19937 + generate_canonical<double> (two words per double), the same
// engine the renderer draws from, so a scene is a pure function of its seed.
struct scene_rng {
  uint32_t x[624];
  uint32_t p = 624;
  explicit scene_rng(uint32_t sd) {
    x[0] = sd;
    for (uint32_t i = 1; i < 624; ++i) x[i] = 1812433253u * (x[i - 1] ^ (x[i - 1] >> 30)) + i;
  }
  uint32_t next() {
    if (p >= 624) {
      for (uint32_t k = 0; k < 624; ++k) {
        uint32_t y = (x[k] & 0x80000000u) | (x[(k + 1) % 624] & 0x7fffffffu);
        x[k] = x[(k + 397) % 624] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
      }
      p = 0;
    }
    uint32_t z = x[p++];
    z ^= z >> 11;
    z ^= (z << 7) & 0x9d2c5680u;
    z ^= (z << 15) & 0xefc60000u;
    z ^= z >> 18;
    return z;
  }
  double canonical() {
    double s = (double)next();
    s = s + (double)next() * 4294967296.0;
    double r = s / 18446744073709551616.0;
    return r >= 1.0 ? 1.0 - 0x1p-53 : r;
  }
  double uniform(double a, double b) { return canonical() * (b - a) + a; }
};

yk_sphere lam(d3 c, double r, d3 alb) {
  yk_sphere s{};
  put(s.center, c);
  s.radius = r;
  put(s.albedo, alb);
  s.material = YK_MATERIAL_LAMBERTIAN;
  return s;
}
yk_sphere met(d3 c, double r, d3 alb, double fuzz) {
  yk_sphere s = lam(c, r, alb);
  s.material = YK_MATERIAL_METAL;
  s.fuzz = fuzz;
  return s;
}
yk_sphere die(d3 c, double r, double ior) {
  yk_sphere s = lam(c, r, {1.0, 1.0, 1.0});
  s.material = YK_MATERIAL_DIELECTRIC;
  s.ior = ior;
  return s;
}

// RTIOW book 1 final scene (configs 3/4), or its dielectric-heavy variant (config 5).
std::vector<yk_sphere> random_scene(uint32_t seed, bool glass_heavy) {
  scene_rng rng(seed);
  std::vector<yk_sphere> w;
  w.push_back(lam({0, -1000, 0}, 1000, {0.5, 0.5, 0.5}));
  const double p_lam = glass_heavy ? 0.3 : 0.8, p_met = glass_heavy ? 0.5 : 0.95;
  for (int a = -11; a < 11; ++a) {
    for (int b = -11; b < 11; ++b) {
      const double choose = rng.canonical();
      const double cx = a + 0.9 * rng.canonical();
      const double cz = b + 0.9 * rng.canonical();
      const d3 center{cx, 0.2, cz};
      const d3 dd = center - d3{4, 0.2, 0};
      if (std::sqrt(dot(dd, dd)) <= 0.9) continue;
      if (choose < p_lam) {
        d3 a1{rng.canonical(), rng.canonical(), rng.canonical()};
        d3 a2{rng.canonical(), rng.canonical(), rng.canonical()};
        w.push_back(lam(center, 0.2, {a1.x * a2.x, a1.y * a2.y, a1.z * a2.z}));
      } else if (choose < p_met) {
        d3 alb{rng.uniform(0.5, 1), rng.uniform(0.5, 1), rng.uniform(0.5, 1)};
        const double fuzz = rng.uniform(0, 0.5);
        w.push_back(met(center, 0.2, alb, fuzz));
      } else {
        w.push_back(die(center, 0.2, 1.5));
      }
    }
  }
  w.push_back(die({0, 1, 0}, 1.0, 1.5));
  if (glass_heavy) {
    w.push_back(die({-4, 1, 0}, 1.0, 1.5));
    w.push_back(die({-4, 1, 0}, -0.9, 1.5));
  } else {
    w.push_back(lam({-4, 1, 0}, 1.0, {0.4, 0.2, 0.1}));
  }
  w.push_back(met({4, 1, 0}, 1.0, {0.7, 0.6, 0.5}, 0.0));
  return w;
}

}  // namespace

extern "C" {

uint32_t yk_image_height_for(uint32_t width) {
  return static_cast<uint32_t>(width / (16.0 / 9.0));  // source.cpp:59-62
}

int yk_camera_reference(yk_camera* out) {
  if (!out) return YK_ERR_INVALID;
  // camera.hpp:16-27, same operations in the same order
  const double aspect_ratio = 16.0 / 9.0;
  const double viewport_height = 2.0;
  const double viewport_width = aspect_ratio * viewport_height;
  const double focal_length = 1.0;
  const d3 h{viewport_width, 0.0, 0.0}, v{0.0, viewport_height, 0.0};
  std::memset(out, 0, sizeof(*out));
  put(out->origin, {0, 0, 0});
  put(out->horizontal, h);
  put(out->vertical, v);
  put(out->lower_left_corner, d3{0, 0, 0} - h / 2 - v / 2 - d3{0, 0, focal_length});
  out->lens_radius = 0.0;
  return YK_OK;
}

int yk_camera_look(yk_camera* out, const double lookfrom[3], const double lookat[3],
                   const double vup[3], double vfov_deg, double aspect, double aperture,
                   double focus_dist) {
  if (!out || !lookfrom || !lookat || !vup || !(vfov_deg > 0) || !(aspect > 0) ||
      !(focus_dist > 0) || !(aperture >= 0))
    return YK_ERR_INVALID;
  const double theta = vfov_deg * M_PI / 180.0;
  const double hh = std::tan(theta / 2);
  const double vh = 2.0 * hh, vw = aspect * vh;
  const d3 from{lookfrom[0], lookfrom[1], lookfrom[2]}, at{lookat[0], lookat[1], lookat[2]};
  const d3 w = unit(from - at);
  const d3 u = unit(cross({vup[0], vup[1], vup[2]}, w));
  const d3 v = cross(w, u);
  const d3 horizontal = u * (focus_dist * vw), vertical = v * (focus_dist * vh);
  std::memset(out, 0, sizeof(*out));
  put(out->origin, from);
  put(out->horizontal, horizontal);
  put(out->vertical, vertical);
  put(out->lower_left_corner, from - horizontal / 2 - vertical / 2 - w * focus_dist);
  put(out->lens_u, u);
  put(out->lens_v, v);
  out->lens_radius = aperture / 2;
  return YK_OK;
}

int yk_scene_build(const char* name, uint32_t seed, yk_sphere* spheres, uint32_t capacity,
                   uint32_t* count, yk_camera* camera) {
  if (!name) return YK_ERR_INVALID;
  const std::string n = name;
  std::vector<yk_sphere> w;
  yk_camera cam{};
  yk_camera_reference(&cam);
  if (n == "ref4") {  // source.cpp:103-112
    w = {lam({0, 0, -1}, 0.5, {0.7, 0.3, 0.3}), lam({0, -100.5, -1}, 100.0, {0.8, 0.8, 0.0}),
         met({-1.0, 0.0, -1.0}, 0.5, {0.8, 0.8, 0.8}, 0), met({1.0, 0.0, -1.0}, 0.5, {0.8, 0.6, 0.2}, 0)};
  } else if (n == "lambert3") {
    w = {lam({0, 0, -1}, 0.5, {0.7, 0.3, 0.3}), lam({0, -100.5, -1}, 100.0, {0.8, 0.8, 0.0}),
         lam({-1.0, 0.0, -1.0}, 0.5, {0.8, 0.8, 0.8})};
  } else if (n == "mixed12") {
    w = {lam({0, -100.5, -1}, 100.0, {0.8, 0.8, 0.0}),  lam({0, 0, -1}, 0.5, {0.1, 0.2, 0.5}),
         met({-1.0, 0.0, -1.0}, 0.5, {0.8, 0.8, 0.8}, 0), met({1.0, 0.0, -1.0}, 0.5, {0.8, 0.6, 0.2}, 0),
         met({0, 0, -1}, 0.5, {0.9, 0.9, 0.9}, 0),       lam({-0.5, 0.6, -1.5}, 0.3, {0.9, 0.1, 0.1}),
         met({0.5, 0.6, -1.5}, 0.3, {0.2, 0.9, 0.2}, 0), lam({0, -0.3, -0.6}, 0.15, {0.2, 0.2, 0.9}),
         met({0.3, 0.1, -0.45}, 0.1, {0.95, 0.95, 0.95}, 0), lam({-0.35, -0.35, -0.7}, 0.12, {0.5, 0.9, 0.5}),
         lam({0, 1.2, -2.5}, 0.6, {0.7, 0.7, 0.7}),      lam({1.0, 0.0, -1.0}, 0.25, {0.3, 0.3, 0.3})};
  } else if (n == "walls2") {
    w = {lam({0, -300.5, -1}, 300.0, {0.9, 0.85, 0.8}), lam({0, 300.5, -1}, 300.0, {0.8, 0.9, 0.95})};
  } else if (n == "rtiow5") {  // config 2: RTIOW three spheres + hollow glass
    w = {lam({0, -100.5, -1}, 100.0, {0.8, 0.8, 0.0}), lam({0, 0, -1}, 0.5, {0.1, 0.2, 0.5}),
         die({-1, 0, -1}, 0.5, 1.5), die({-1, 0, -1}, -0.4, 1.5),
         met({1, 0, -1}, 0.5, {0.8, 0.6, 0.2}, 0.0)};
    const double f[3] = {-2, 2, 1}, a[3] = {0, 0, -1}, up[3] = {0, 1, 0};
    yk_camera_look(&cam, f, a, up, 20.0, 16.0 / 9.0, 0.0, 1.0);
  } else if (n == "final" || n == "glass") {  // configs 3/4 and 5
    w = random_scene(seed, n == "glass");
    const double f[3] = {13, 2, 3}, a[3] = {0, 0, 0}, up[3] = {0, 1, 0};
    yk_camera_look(&cam, f, a, up, 20.0, 16.0 / 9.0, 0.1, 10.0);
  } else {
    return YK_ERR_INVALID;
  }
  if (count) *count = (uint32_t)w.size();
  if (camera) *camera = cam;
  if (spheres) {
    if (capacity < w.size()) return YK_ERR_INVALID;
    std::memcpy(spheres, w.data(), w.size() * sizeof(yk_sphere));
  }
  return YK_OK;
}

}  // extern "C"

// ---- scene files -------------------------------------------------------------------------
// Text, one record per line, numbers as %.17g (every double round-trips exactly):
//   yk-scene 1
//   camera <origin 3> <lower_left_corner 3> <horizontal 3> <vertical 3> <lens_u 3> <lens_v 3> <lens_radius>
//   sphere <lambertian|metal|dielectric> <cx cy cz> <radius> <albedo r g b> <fuzz> <ior>
// '#' starts a comment line.  The spheres keep file order = tuple order (it defines rec.id).
namespace {
const char* kind_name(uint32_t k) {
  return k == YK_MATERIAL_LAMBERTIAN ? "lambertian" : k == YK_MATERIAL_METAL ? "metal" : "dielectric";
}
}  // namespace

int yk_scene_write(const char* path, const yk_sphere* spheres, uint32_t count, const yk_camera* camera) {
  if (!path || !camera || (count && !spheres)) return YK_ERR_INVALID;
  FILE* f = std::fopen(path, "w");
  if (!f) return YK_ERR_INVALID;
  std::fprintf(f, "yk-scene 1\n# %u spheres; tuple order\ncamera", count);
  const double* cv[6] = {camera->origin, camera->lower_left_corner, camera->horizontal,
                         camera->vertical, camera->lens_u, camera->lens_v};
  for (const double* v : cv) std::fprintf(f, " %.17g %.17g %.17g", v[0], v[1], v[2]);
  std::fprintf(f, " %.17g\n", camera->lens_radius);
  for (uint32_t i = 0; i < count; ++i) {
    const yk_sphere& s = spheres[i];
    std::fprintf(f, "sphere %s %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", kind_name(s.material),
                 s.center[0], s.center[1], s.center[2], s.radius, s.albedo[0], s.albedo[1], s.albedo[2],
                 s.fuzz, s.ior);
  }
  const bool ok = std::ferror(f) == 0;
  return (std::fclose(f) == 0 && ok) ? YK_OK : YK_ERR_INVALID;
}

int yk_scene_read(const char* path, yk_sphere* spheres, uint32_t capacity, uint32_t* count, yk_camera* camera) {
  if (!path) return YK_ERR_INVALID;
  FILE* f = std::fopen(path, "r");
  if (!f) return YK_ERR_INVALID;
  std::vector<yk_sphere> w;
  yk_camera cam{};
  bool have_header = false, have_camera = false, bad = false;
  char line[1024];
  while (!bad && std::fgets(line, sizeof line, f)) {
    char word[32] = {0};
    if (line[0] == '#' || std::sscanf(line, "%31s", word) != 1) continue;
    const std::string wd = word;
    if (wd == "yk-scene") {
      int v = 0;
      bad = std::sscanf(line, "%*s %d", &v) != 1 || v != 1;
      have_header = true;
    } else if (wd == "camera") {
      double* cv[6] = {cam.origin, cam.lower_left_corner, cam.horizontal, cam.vertical, cam.lens_u, cam.lens_v};
      const char* p = line + 6;
      int used = 0;
      for (double* v : cv)
        for (int k = 0; k < 3 && !bad; ++k) {
          bad = std::sscanf(p, "%lf%n", &v[k], &used) != 1;
          p += used;
        }
      bad = bad || std::sscanf(p, "%lf", &cam.lens_radius) != 1;
      have_camera = true;
    } else if (wd == "sphere") {
      yk_sphere s;
      std::memset(&s, 0, sizeof s);
      char kind[32] = {0};
      bad = std::sscanf(line, "%*s %31s %lf %lf %lf %lf %lf %lf %lf %lf %lf", kind, &s.center[0], &s.center[1],
                        &s.center[2], &s.radius, &s.albedo[0], &s.albedo[1], &s.albedo[2], &s.fuzz, &s.ior) != 10;
      const std::string k = kind;
      if (k == "lambertian") s.material = YK_MATERIAL_LAMBERTIAN;
      else if (k == "metal") s.material = YK_MATERIAL_METAL;
      else if (k == "dielectric") s.material = YK_MATERIAL_DIELECTRIC;
      else bad = true;
      w.push_back(s);
    } else {
      bad = true;
    }
  }
  std::fclose(f);
  if (bad || !have_header || !have_camera) return YK_ERR_INVALID;
  if (count) *count = (uint32_t)w.size();
  if (camera) *camera = cam;
  if (spheres) {
    if (capacity < w.size()) return YK_ERR_INVALID;
    if (!w.empty()) std::memcpy(spheres, w.data(), w.size() * sizeof(yk_sphere));
  }
  return YK_OK;
}

