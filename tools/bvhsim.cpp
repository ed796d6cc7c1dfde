// tools/bvhsim.cpp — CPU model of the kernel's BVH traversal, for choosing BVH build options.
//
// Generates the segment rays of a path-traced image of a named scene (approximate shading:
// the ray DISTRIBUTION is what matters here, not exact colours), replays the kernel's
// traversal on them (float slabs, ordered descent, U* from the hit bound) and prints per-ray
// visit statistics plus the expected maximum over random groups of 64 rays — the number of
// loop trips a wave pays in the while-while loop.
//   build: make -C tools bvhsim      run: tools/bvhsim final 42 [leaf bins]
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "../include/ykgpu.h"
#include "../uecraytracing_amd/csrc/yk_bvh.hpp"

struct V {
  double x, y, z;
};
static V add(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V sub(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static V mul(V a, double s) { return {a.x * s, a.y * s, a.z * s}; }
static double dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static V unit(V a) { return mul(a, 1.0 / std::sqrt(dot(a, a))); }
static V ld(const double* p) { return {p[0], p[1], p[2]}; }

struct Stats {
  uint32_t nodes = 0, leaves = 0, tests = 0;
};

struct Sim {
  std::vector<yk_sphere> sph;
  ykbvh::Built bvh;
  std::vector<uint32_t> leaf_ids;

  // exact-ish closest hit (double), returns id or -1
  int hit_exact(V o, V d, double& t) const {
    int best = -1;
    t = INFINITY;
    for (size_t i = 0; i < sph.size(); ++i) {
      V oc = sub(o, ld(sph[i].center));
      double a = dot(d, d), hb = dot(oc, d), c = dot(oc, oc) - sph[i].radius * sph[i].radius;
      double disc = hb * hb - a * c;
      if (disc < 0) continue;
      double sq = std::sqrt(disc), r = (-hb - sq) / a;
      if (r < 0.001) r = (-hb + sq) / a;
      if (r < 0.001) continue;
      if (r <= t) { t = r; best = (int)i; }
    }
    return best;
  }

  Stats traverse(V o, V d) const {
    Stats st;
    auto rcp = [](float x) { return std::fabs(x) > 1e-30f ? 1.0f / x : std::copysign(1e30f, x); };
    const float ix = rcp((float)d.x), iy = rcp((float)d.y), iz = rcp((float)d.z);
    const float oix = (float)o.x * ix, oiy = (float)o.y * iy, oiz = (float)o.z * iz;
    const double a = dot(d, d);
    double ustar = INFINITY;
    float uf = INFINITY;
    int32_t stack[64];
    int sp = 0;
    int32_t node = bvh.root;
    for (;;) {
      if (node >= 0) {
        ++st.nodes;
        const ykbvh::Node& nd = bvh.nodes[node];
        float tn[2], tf[2];
        for (int k = 0; k < 2; ++k) {
          float ax = std::fma(nd.lo_x[k], ix, -oix), bx = std::fma(nd.hi_x[k], ix, -oix);
          float ay = std::fma(nd.lo_y[k], iy, -oiy), by = std::fma(nd.hi_y[k], iy, -oiy);
          float az = std::fma(nd.lo_z[k], iz, -oiz), bz = std::fma(nd.hi_z[k], iz, -oiz);
          float n0 = std::max(std::max(std::min(ax, bx), std::min(ay, by)), std::min(az, bz));
          float f0 = std::min(std::min(std::max(ax, bx), std::max(ay, by)), std::max(az, bz));
          tn[k] = n0 - std::fabs(n0) * 0x1p-20f;
          tf[k] = f0 + std::fabs(f0) * 0x1p-20f;
        }
        bool h0 = tn[0] <= tf[0] && tf[0] >= 0.001f && tn[0] <= uf;
        bool h1 = tn[1] <= tf[1] && tf[1] >= 0.001f && tn[1] <= uf;
        if (h0 && h1) {
          bool f = tn[0] <= tn[1];
          stack[sp++] = f ? nd.child[1] : nd.child[0];
          node = f ? nd.child[0] : nd.child[1];
          continue;
        }
        if (h0 || h1) {
          node = h0 ? nd.child[0] : nd.child[1];
          continue;
        }
      } else {
        ++st.leaves;
        uint32_t v = ~(uint32_t)node, first = v >> 4, cnt = v & 15u;
        for (uint32_t k = 0; k < cnt; ++k) {
          ++st.tests;
          const yk_sphere& s = sph[leaf_ids[first + k]];
          V oc = sub(o, ld(s.center));
          double hb = dot(oc, d), c = dot(oc, oc) - s.radius * s.radius;
          double disc = hb * hb - a * c;
          if (disc < 0) continue;
          double sq = std::sqrt(disc), r1 = (-hb - sq) / a, r2 = (-hb + sq) / a;
          double ub = r1 >= 0.001 ? r1 : (r2 >= 0.001 ? r2 : INFINITY);
          if (ub < ustar) { ustar = ub; uf = (float)ub * (1 + 0x1p-20f); }
        }
      }
      if (sp == 0) break;
      node = stack[--sp];
    }
    return st;
  }
};

int main(int argc, char** argv) {
  const char* scene = argc > 1 ? argv[1] : "final";
  uint32_t seed = argc > 2 ? atoi(argv[2]) : 42;
  ykbvh::Options opt;
  if (argc > 3) opt.max_leaf = atoi(argv[3]);
  if (argc > 4) opt.bins = atoi(argv[4]);
  Sim sim;
  uint32_t n = 0;
  yk_camera cam;
  yk_scene_build(scene, seed, nullptr, 0, &n, &cam);
  sim.sph.resize(n);
  yk_scene_build(scene, seed, sim.sph.data(), n, &n, nullptr);
  std::vector<double> c(3 * n), r(n);
  for (uint32_t i = 0; i < n; ++i) {
    for (int k = 0; k < 3; ++k) c[3 * i + k] = sim.sph[i].center[k];
    r[i] = sim.sph[i].radius;
  }
  sim.bvh = ykbvh::build(c.data(), r.data(), n, 13.0, opt);
  sim.leaf_ids = sim.bvh.order;
  // rays: 192x108 px, 2 spp, simple shading
  std::mt19937_64 rng(1);
  std::uniform_real_distribution<double> U(0, 1);
  std::vector<Stats> rays;
  const int W = 192, H = 108;
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x)
      for (int s = 0; s < 2; ++s) {
        double u = (x + U(rng)) / W, v = (H - y - 1 + U(rng)) / H;
        V o = ld(cam.origin);
        V d = sub(add(add(ld(cam.lower_left_corner), mul(ld(cam.horizontal), u)), mul(ld(cam.vertical), v)), o);
        for (int depth = 0; depth < 50; ++depth) {
          rays.push_back(sim.traverse(o, d));
          double t;
          int id = sim.hit_exact(o, d, t);
          if (id < 0) break;
          const yk_sphere& sp = sim.sph[id];
          V p = add(o, mul(d, t));
          V nrm = mul(sub(p, ld(sp.center)), 1.0 / sp.radius);
          bool front = dot(d, nrm) < 0;
          if (!front) nrm = mul(nrm, -1);
          if (sp.material == YK_MATERIAL_LAMBERTIAN) {
            V q{U(rng) * 2 - 1, U(rng) * 2 - 1, U(rng) * 2 - 1};
            d = add(nrm, unit(q));
          } else if (sp.material == YK_MATERIAL_METAL) {
            V ud = unit(d);
            d = sub(ud, mul(nrm, 2 * dot(ud, nrm)));
            if (sp.fuzz > 0) d = add(d, mul(unit(V{U(rng) - .5, U(rng) - .5, U(rng) - .5}), sp.fuzz * U(rng)));
            if (dot(d, nrm) <= 0) break;
          } else {
            V ud = unit(d);
            double ratio = front ? 1 / sp.ior : sp.ior, ct = std::min(-dot(ud, nrm), 1.0);
            double stt = std::sqrt(1 - ct * ct);
            if (ratio * stt > 1 || U(rng) < 0.1) d = sub(ud, mul(nrm, 2 * dot(ud, nrm)));
            else {
              V perp = mul(add(ud, mul(nrm, ct)), ratio);
              d = add(perp, mul(nrm, -std::sqrt(std::fabs(1 - dot(perp, perp)))));
            }
          }
          o = p;
        }
      }
  auto steps = [](const Stats& s) { return s.nodes + s.leaves; };
  std::vector<uint32_t> st(rays.size());
  double sum_n = 0, sum_l = 0, sum_t = 0;
  for (size_t i = 0; i < rays.size(); ++i) {
    st[i] = steps(rays[i]);
    sum_n += rays[i].nodes;
    sum_l += rays[i].leaves;
    sum_t += rays[i].tests;
  }
  std::vector<uint32_t> sorted = st;
  std::sort(sorted.begin(), sorted.end());
  auto pct = [&](double q) { return sorted[(size_t)(q * (sorted.size() - 1))]; };
  // expected max over random groups of 64
  std::vector<uint32_t> perm = st;
  std::shuffle(perm.begin(), perm.end(), rng);
  double sum_max = 0, sum_mean = 0;
  size_t groups = perm.size() / 64;
  for (size_t g = 0; g < groups; ++g) {
    uint32_t mx = 0;
    double mn = 0;
    for (int k = 0; k < 64; ++k) {
      mx = std::max(mx, perm[g * 64 + k]);
      mn += perm[g * 64 + k];
    }
    sum_max += mx;
    sum_mean += mn / 64;
  }
  const size_t R = rays.size();
  printf("%s n=%u nodes=%zu depth=%u leaf<=%u bins=%d | rays %zu: nodes %.2f leaves %.2f tests %.2f | steps p50 %u p90 %u p99 %u max %u | wave E[max]/E[mean] %.2f/%.2f = %.2f\n",
         scene, n, sim.bvh.nodes.size(), sim.bvh.depth, opt.max_leaf, opt.bins, R, sum_n / R, sum_l / R,
         sum_t / R, pct(0.5), pct(0.9), pct(0.99), sorted.back(), sum_max / groups, sum_mean / groups,
         sum_max / sum_mean);
  return 0;
}
