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

// ---- 4-wide model: the binary tree collapsed (each slot's interior child replaced by its two
// children, largest surface area first) and the kernel's while-while loop replayed in lockstep
struct Wide {
  float lo[4][3], hi[4][3];
  int32_t code[4];  // >= 0: wide node index; < 0: leaf code; INT32_MIN: empty
  int n;
};

// the slot chosen for expansion (round 6 exploration): 0 the largest area (the library's rule),
// 1 the largest area x leaves below, 2 the largest area x (leaves below)^0.5
static int g_collapse = 0;
static std::vector<uint32_t> g_leaves;  // leaves under each binary node
static uint32_t count_leaves(const ykbvh::Built& b, int32_t code) {
  if (code < 0) return 1;
  if (g_leaves[code]) return g_leaves[code];
  return g_leaves[code] = count_leaves(b, b.nodes[code].child[0]) + count_leaves(b, b.nodes[code].child[1]);
}
static void collapse(const ykbvh::Built& b, std::vector<Wide>& out, int32_t code, int width) {
  // code >= 0: binary node index
  struct E { float lo[3], hi[3]; int32_t code; };
  std::vector<E> ents;
  const ykbvh::Node& nd = b.nodes[code];
  for (int k = 0; k < 2; ++k)
    ents.push_back({{nd.lo_x[k], nd.lo_y[k], nd.lo_z[k]}, {nd.hi_x[k], nd.hi_y[k], nd.hi_z[k]}, nd.child[k]});
  auto area = [](const E& e) {
    float dx = e.hi[0] - e.lo[0], dy = e.hi[1] - e.lo[1], dz = e.hi[2] - e.lo[2];
    return dx * dy + dy * dz + dz * dx;
  };
  auto score = [&](const E& e) {
    const double a = area(e), nl = e.code >= 0 ? count_leaves(b, e.code) : 1;
    return g_collapse == 1 ? a * nl : g_collapse == 2 ? a * std::sqrt(nl) : a;
  };
  while ((int)ents.size() < width) {
    int best = -1;
    for (size_t i = 0; i < ents.size(); ++i)
      if (ents[i].code >= 0 && (best < 0 || score(ents[i]) > score(ents[best]))) best = (int)i;
    if (best < 0) break;
    const ykbvh::Node& c = b.nodes[ents[best].code];
    E e0{{c.lo_x[0], c.lo_y[0], c.lo_z[0]}, {c.hi_x[0], c.hi_y[0], c.hi_z[0]}, c.child[0]};
    E e1{{c.lo_x[1], c.lo_y[1], c.lo_z[1]}, {c.hi_x[1], c.hi_y[1], c.hi_z[1]}, c.child[1]};
    ents[best] = e0;
    ents.push_back(e1);
  }
  const size_t me = out.size();
  out.push_back(Wide{});
  Wide w{};
  w.n = (int)ents.size();
  for (int k = 0; k < 4; ++k) {
    if (k < w.n) {
      for (int a = 0; a < 3; ++a) { w.lo[k][a] = ents[k].lo[a]; w.hi[k][a] = ents[k].hi[a]; }
      if (ents[k].code >= 0) {
        w.code[k] = (int32_t)out.size();
        collapse(b, out, ents[k].code, width);
      } else {
        w.code[k] = ents[k].code;
      }
    } else {
      w.code[k] = INT32_MIN;
    }
  }
  out[me] = w;
}

// per-lane traversal state machine for the lockstep wave model
struct Lane {
  float ix, iy, iz, oix, oiy, oiz;
  double ustar;
  float uf;
  int32_t stack[64];
  int sp;
  int32_t node;
  bool done;
  bool at_leaf;
  V o, d;
  double a;
};

int main(int argc, char** argv) {
  const char* scene = argc > 1 ? argv[1] : "final";
  uint32_t seed = argc > 2 ? atoi(argv[2]) : 42;
  ykbvh::Options opt;
  if (argc > 3) opt.max_leaf = atoi(argv[3]);
  if (argc > 4) opt.bins = atoi(argv[4]);
  opt.all_axes = argc > 5 ? atoi(argv[5]) != 0 : true;  // (the FP64 tree: all three axes)
  if (argc > 6) g_collapse = atoi(argv[6]);
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
  std::vector<std::pair<V, V>> seg;
  const int W = 192, H = 108;
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x)
      for (int s = 0; s < 2; ++s) {
        double u = (x + U(rng)) / W, v = (H - y - 1 + U(rng)) / H;
        V o = ld(cam.origin);
        V d = sub(add(add(ld(cam.lower_left_corner), mul(ld(cam.horizontal), u)), mul(ld(cam.vertical), v)), o);
        for (int depth = 0; depth < 50; ++depth) {
          rays.push_back(sim.traverse(o, d));
          seg.push_back({o, d});
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
  // ---- lockstep wave model: binary vs 4-wide, while-while loop as compiled
  std::vector<Wide> wide;
  g_leaves.assign(sim.bvh.nodes.size(), 0);
  if (sim.bvh.root >= 0) collapse(sim.bvh, wide, sim.bvh.root, 4);
  std::vector<size_t> idx(seg.size());
  for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
  std::shuffle(idx.begin(), idx.end(), rng);
  auto leaf_test = [&](Lane& L, int32_t code) {
    uint32_t v = ~(uint32_t)code, first = v >> 4, cnt = v & 15u;
    for (uint32_t k = 0; k < cnt; ++k) {
      const yk_sphere& s = sim.sph[sim.leaf_ids[first + k]];
      V oc = sub(L.o, ld(s.center));
      double hb = dot(oc, L.d), c = dot(oc, oc) - s.radius * s.radius;
      double disc = hb * hb - L.a * c;
      if (disc < 0) continue;
      double sq = std::sqrt(disc), r1 = (-hb - sq) / L.a, r2 = (-hb + sq) / L.a;
      double ub = r1 >= 0.001 ? r1 : (r2 >= 0.001 ? r2 : INFINITY);
      if (ub < L.ustar) { L.ustar = ub; L.uf = (float)ub * (1 + 0x1p-20f); }
    }
    return cnt;
  };
  for (int width : {2, 4, 5, 6, 7}) {
    double w_inner = 0, w_leaf = 0, w_outer = 0, l_inner = 0, l_leafiters = 0;
    int max_sp = 0;
    std::vector<size_t> sp_hist(80, 0);
    size_t nw = 0;
    for (size_t g = 0; g + 64 <= idx.size(); g += 64) {
      std::vector<Lane> lanes(64);
      for (int k = 0; k < 64; ++k) {
        Lane& L = lanes[k];
        V o = seg[idx[g + k]].first, d = seg[idx[g + k]].second;
        auto rcp = [](float x) { return std::fabs(x) > 1e-30f ? 1.0f / x : std::copysign(1e30f, x); };
        L.ix = rcp((float)d.x); L.iy = rcp((float)d.y); L.iz = rcp((float)d.z);
        L.oix = (float)o.x * L.ix; L.oiy = (float)o.y * L.iy; L.oiz = (float)o.z * L.iz;
        L.ustar = INFINITY; L.uf = INFINITY; L.sp = 0; L.done = false; L.at_leaf = false;
        L.o = o; L.d = d; L.a = dot(d, d);
        L.node = width == 2 ? sim.bvh.root : (sim.bvh.root >= 0 ? 0 : sim.bvh.root);
      }
      auto slab = [&](Lane& L, const float* lo, const float* hi, float& tn) {
        float ax = std::fma(lo[0], L.ix, -L.oix), bx = std::fma(hi[0], L.ix, -L.oix);
        float ay = std::fma(lo[1], L.iy, -L.oiy), by = std::fma(hi[1], L.iy, -L.oiy);
        float az = std::fma(lo[2], L.iz, -L.oiz), bz = std::fma(hi[2], L.iz, -L.oiz);
        float n0 = std::max(std::max(std::min(ax, bx), std::min(ay, by)), std::min(az, bz));
        float f0 = std::min(std::min(std::max(ax, bx), std::max(ay, by)), std::max(az, bz));
        tn = std::max(n0 - std::fabs(n0) * 0x1p-20f, 0.001f);
        float tf = std::min(f0 + std::fabs(f0) * 0x1p-20f, L.uf);
        return tn <= tf;
      };
      // one interior step; returns false when the lane leaves the inner loop (leaf / nothing hit)
      auto step = [&](Lane& L) -> bool {
        if (width == 2) {
          const ykbvh::Node& nd = sim.bvh.nodes[L.node];
          float tn[2];
          bool h[2];
          for (int k = 0; k < 2; ++k) {
            float lo[3] = {nd.lo_x[k], nd.lo_y[k], nd.lo_z[k]}, hi[3] = {nd.hi_x[k], nd.hi_y[k], nd.hi_z[k]};
            h[k] = slab(L, lo, hi, tn[k]);
          }
          if (h[0] && h[1]) {
            bool f = tn[0] <= tn[1];
            L.stack[L.sp++] = f ? nd.child[1] : nd.child[0];
            L.node = f ? nd.child[0] : nd.child[1];
          } else if (h[0] || h[1]) {
            L.node = h[0] ? nd.child[0] : nd.child[1];
          } else {
            return false;
          }
        } else {
          const Wide& w = wide[L.node];
          std::pair<float, int32_t> hits[4];
          int nh = 0;
          for (int k = 0; k < w.n; ++k) {
            float tn;
            if (slab(L, w.lo[k], w.hi[k], tn)) hits[nh++] = {tn, w.code[k]};
          }
          if (!nh) return false;
          if (width == 6 || width == 7) {
            // no distance ordering: visit one hit slot, push the others (child order; width 7:
            // the order reversed when the ray runs along +axis of the node's slot spread)
            bool rev = false;
            if (width == 7) {
              int ax = 0; float best = -1;
              for (int a = 0; a < 3; ++a) {
                float c0 = w.lo[0][a] + w.hi[0][a], c1 = w.lo[w.n - 1][a] + w.hi[w.n - 1][a];
                if (std::fabs(c1 - c0) > best) { best = std::fabs(c1 - c0); ax = a; }
              }
              float dd = ax == 0 ? (float)L.d.x : ax == 1 ? (float)L.d.y : (float)L.d.z;
              float c0 = w.lo[0][ax] + w.hi[0][ax], c1 = w.lo[w.n - 1][ax] + w.hi[w.n - 1][ax];
              rev = (dd > 0) == (c1 > c0);  // slots already near-to-far: visit the first
            }
            if (rev) std::reverse(hits, hits + nh);
            // visit the LAST of hits[] first, push the rest in order (the stack pops hits[nh-2] next)
            for (int k = 0; k < nh - 1; ++k) L.stack[L.sp++] = hits[k].second;
            L.node = hits[nh - 1].second;
            max_sp = std::max(max_sp, L.sp);
            return L.node >= 0;
          }
          if (width == 4) {
            std::sort(hits, hits + nh, [](auto& x, auto& y) { return x.first < y.first; });
          } else {  // width 5 = 4-wide, nearest first, the rest pushed in child order
            int b = 0;
            for (int k = 1; k < nh; ++k) if (hits[k].first < hits[b].first) b = k;
            std::swap(hits[0], hits[b]);
          }
          for (int k = nh - 1; k >= 1; --k) L.stack[L.sp++] = hits[k].second;
          L.node = hits[0].second;
          max_sp = std::max(max_sp, L.sp);
          sp_hist[L.sp]++;
        }
        return L.node >= 0;
      };
      for (;;) {
        bool any = false;
        for (auto& L : lanes) any |= !L.done;
        if (!any) break;
        // inner loop over interior nodes
        std::vector<bool> in(64);
        for (int k = 0; k < 64; ++k) in[k] = !lanes[k].done && lanes[k].node >= 0;
        for (;;) {
          int active = 0;
          for (int k = 0; k < 64; ++k)
            if (in[k]) { ++active; in[k] = step(lanes[k]); }
          if (!active) break;
          w_inner += 1;
          l_inner += active;
        }
        // leaf + pop
        uint32_t mx = 0, act = 0;
        for (auto& L : lanes) {
          if (L.done) continue;
          ++act;
          if (L.node < 0) { uint32_t c = leaf_test(L, L.node); mx = std::max(mx, c); l_leafiters += c; }
          if (L.sp == 0) L.done = true;
          else L.node = L.stack[--L.sp];
        }
        w_leaf += mx;
        w_outer += 1;
      }
      ++nw;
    }
    printf("width %d: per wave-segment: inner iters %.1f (lane util %.0f%%), leaf iters %.1f, outer rounds %.1f; wide nodes %zu max sp %d",
           width, w_inner / nw, 100.0 * l_inner / (64.0 * w_inner), w_leaf / nw, w_outer / nw, wide.size(), max_sp);
    for (int k = 8; k < 20; ++k) printf(" [%d]%zu", k, sp_hist[k]);
    printf("\n");
  }
  return 0;
}
