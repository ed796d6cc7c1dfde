// tools/loopsim.cpp — lockstep wave model of the FP64 kernel's traversal LOOP SHAPE, on the
// device's own 4-wide tree (ykbvh::wide_nodes) and the kernel's visit order (last entered slot
// next, the others pushed in slot order).  It compares loop structures by the wave-level work
// they issue, which is what the render pays for:
//   ifelse  — the shipped loop: per trip a lane visits an inner node OR tests a leaf;
//   postpone — per trip a lane visits an inner node AND tests one postponed leaf (a leaf met
//              while traversing is parked in a register and the traversal pops on).
// Costs per wave trip are VALU-instruction weights of the blocks (measured from the ISA, command
// line): visit, leaf discriminant, the disc >= 0 tail, loop overhead.
//   build: g++ -O2 -std=c++17 -Iinclude tools/loopsim.cpp uecraytracing_amd/csrc/yk_bvh.cpp \
//          uecraytracing_amd/csrc/yk_host.cpp -o /tmp/loopsim
//   run:   /tmp/loopsim final 42 [leaf] [c_visit c_leaf c_disc c_trip frac]
//   env:   YKSIM_BINS=n (SAH bins), YKSIM_ALLAXES=1 (SAH over all axes), YKSIM_WIDTH=n (an n-wide
//          tree, n <= 8, in the if/else loop: wave-level visit and leaf blocks per segment)
// The pool models (a wave-wide LIFO of (ray, node) pairs) and the speculative variant count wave
// trips and blocks only; their measured kernels were slower or neutral, because the
// node loop is bound by LDS latency and trip count, which these weights do not price.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <deque>
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

constexpr int32_t kDone = INT32_MIN;  // no node (stack empty)
constexpr int32_t kNone = 0;          // no postponed leaf (leaf codes are negative)

struct Lane {
  V o, d;
  double a, ustar = INFINITY;
  float ix, iy, iz, uf = INFINITY;
  std::vector<int32_t> stk;
  int32_t node = 0, pend = kNone;
  bool done = false;
};

struct Model {
  std::vector<yk_sphere> sph;
  std::vector<ykbvh::WideNode> wide;
  std::vector<uint32_t> order;
  int32_t root = 0;

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
  // one interior visit: returns the next node (or kDone after an empty pop)
  void visit(Lane& L) const {
    const ykbvh::WideNode& w = wide[L.node / (int32_t)sizeof(ykbvh::WideNode)];
    const float c = 1.0f + 0x1p-17f;
    bool hk[4];
    for (int k = 0; k < 4; ++k) {
      const int sx = L.ix < 0 ? 4 : 0, sy = L.iy < 0 ? 4 : 0, sz = L.iz < 0 ? 4 : 0;
      const float nx = std::fma(w.x[sx + k], L.ix, -(float)L.o.x * L.ix);
      const float fx = std::fma(w.x[sx + 4 + k], L.ix * c, -((float)L.o.x * L.ix * c));
      const float ny = std::fma(w.y[sy + k], L.iy, -(float)L.o.y * L.iy);
      const float fy = std::fma(w.y[sy + 4 + k], L.iy * c, -((float)L.o.y * L.iy * c));
      const float nz = std::fma(w.z[sz + k], L.iz, -(float)L.o.z * L.iz);
      const float fz = std::fma(w.z[sz + 4 + k], L.iz * c, -((float)L.o.z * L.iz * c));
      const float tn = std::max(std::max(std::max(nx, ny), nz), 0.001f * (1 - 0x1p-17f));
      const float tf = std::min(std::min(std::min(fx, fy), fz), L.uf);
      hk[k] = tn <= tf;
    }
    int last = -1;
    for (int k = 0; k < 4; ++k)
      if (hk[k]) last = k;
    if (last < 0) {
      pop(L);
      return;
    }
    for (int k = 0; k < last; ++k)
      if (hk[k]) L.stk.push_back(w.child[k]);
    L.node = w.child[last];
  }
  static void pop(Lane& L) {
    if (L.stk.empty()) {
      L.node = kDone;
    } else {
      L.node = L.stk.back();
      L.stk.pop_back();
    }
  }
  // leaf test: returns (spheres tested, disc >= 0 count)
  std::pair<int, int> leaf(Lane& L, int32_t code) const {
    const uint32_t v = ~(uint32_t)code, first = v >> 4, cnt = v & 15u;
    int dpos = 0;
    for (uint32_t k = 0; k < cnt; ++k) {
      const yk_sphere& s = sph[order[first + k]];
      V oc = sub(L.o, ld(s.center));
      double hb = dot(oc, L.d), cc = dot(oc, oc) - s.radius * s.radius;
      double disc = hb * hb - L.a * cc;
      if (disc < 0) continue;
      ++dpos;
      double sq = std::sqrt(disc), r1 = (-hb - sq) / L.a, r2 = (-hb + sq) / L.a;
      double ub = r1 >= 0.001 ? r1 : (r2 >= 0.001 ? r2 : INFINITY);
      if (ub < L.ustar) { L.ustar = ub; L.uf = (float)ub * (1 + 0x1p-18f); }
    }
    return {(int)cnt, dpos};
  }
};

// ---- N-wide model (YKSIM_WIDTH=N, N <= 8): the binary tree collapsed greedily (largest surface
// area first, as ykbvh::wide_nodes) to N slots per node; the same if/else loop per lane
struct WideN {
  float lo[8][3], hi[8][3];
  int32_t code[8];  // >= 0: node index, < 0: leaf code
  int n;
};
static void collapse_n(const ykbvh::Built& b, std::vector<WideN>& out, int32_t code, int width) {
  struct E { float lo[3], hi[3]; int32_t code; };
  auto ent = [&](const ykbvh::Node& nd, int k) {
    return E{{nd.lo_x[k], nd.lo_y[k], nd.lo_z[k]}, {nd.hi_x[k], nd.hi_y[k], nd.hi_z[k]}, nd.child[k]};
  };
  std::vector<E> ents = {ent(b.nodes[code], 0), ent(b.nodes[code], 1)};
  auto area = [](const E& e) {
    float dx = e.hi[0] - e.lo[0], dy = e.hi[1] - e.lo[1], dz = e.hi[2] - e.lo[2];
    return dx * dy + dy * dz + dz * dx;
  };
  while ((int)ents.size() < width) {
    int best = -1;
    for (size_t i = 0; i < ents.size(); ++i)
      if (ents[i].code >= 0 && (best < 0 || area(ents[i]) > area(ents[best]))) best = (int)i;
    if (best < 0) break;
    const ykbvh::Node& c = b.nodes[ents[best].code];
    ents[best] = ent(c, 0);
    ents.insert(ents.begin() + best + 1, ent(c, 1));
  }
  const size_t me = out.size();
  out.push_back(WideN{});
  WideN w{};
  w.n = (int)ents.size();
  for (int k = 0; k < w.n; ++k) {
    for (int a = 0; a < 3; ++a) { w.lo[k][a] = ents[k].lo[a]; w.hi[k][a] = ents[k].hi[a]; }
    if (ents[k].code >= 0) {
      w.code[k] = (int32_t)out.size();
      collapse_n(b, out, ents[k].code, width);
    } else {
      w.code[k] = ents[k].code;
    }
  }
  out[me] = w;
}

int main(int argc, char** argv) {
  const char* scene = argc > 1 ? argv[1] : "final";
  uint32_t seed = argc > 2 ? atoi(argv[2]) : 42;
  ykbvh::Options opt;
  if (argc > 3) opt.max_leaf = atoi(argv[3]);
  if (const char* e = getenv("YKSIM_BINS")) opt.bins = atoi(e);
  if (getenv("YKSIM_ALLAXES")) opt.all_axes = true;
  const double c_visit = argc > 4 ? atof(argv[4]) : 53, c_leaf = argc > 5 ? atof(argv[5]) : 20,
               c_disc = argc > 6 ? atof(argv[6]) : 40, c_trip = argc > 7 ? atof(argv[7]) : 10,
               frac = argc > 8 ? atof(argv[8]) : 1.0;
  Model M;
  uint32_t n = 0;
  yk_camera cam;
  yk_scene_build(scene, seed, nullptr, 0, &n, &cam);
  M.sph.resize(n);
  yk_scene_build(scene, seed, M.sph.data(), n, &n, nullptr);
  std::vector<double> c(3 * n), r(n);
  for (uint32_t i = 0; i < n; ++i) {
    for (int k = 0; k < 3; ++k) c[3 * i + k] = M.sph[i].center[k];
    r[i] = M.sph[i].radius;
  }
  double ext = 0;
  for (int k = 0; k < 3; ++k) ext = std::max(ext, std::fabs(cam.origin[k]));
  const ykbvh::Built b = ykbvh::build(c.data(), r.data(), n, ext, opt);
  uint32_t wd = 0;
  M.wide = ykbvh::wide_nodes(b, &M.root, &wd);
  M.order = b.order;
  // segment rays of a 192x108x2 path-traced image (approximate shading: the distribution matters)
  std::mt19937_64 rng(1);
  std::uniform_real_distribution<double> U(0, 1);
  std::vector<std::pair<V, V>> seg;
  std::vector<int> seg_depth;
  const int W = getenv("YKSIM_W") ? atoi(getenv("YKSIM_W")) : 192, H = W * 9 / 16;
  const int SPP = getenv("YKSIM_SPP") ? atoi(getenv("YKSIM_SPP")) : 2;
  for (int y = 0; y < H; ++y)
    for (int x = 0; x < W; ++x)
      for (int s = 0; s < SPP; ++s) {
        double u = (x + U(rng)) / W, v = (H - y - 1 + U(rng)) / H;
        V o = ld(cam.origin);
        V d = sub(add(add(ld(cam.lower_left_corner), mul(ld(cam.horizontal), u)), mul(ld(cam.vertical), v)), o);
        for (int depth = 0; depth < 50; ++depth) {
          seg.push_back({o, d});
          seg_depth.push_back(depth);
          double t;
          int id = M.hit_exact(o, d, t);
          if (id < 0) break;
          const yk_sphere& sp = M.sph[id];
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
  std::vector<size_t> idx(seg.size());
  for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
  // YKSIM_SECONDARY=1: the bounce segments only (what the render loop would run if the first
  // segment of every sample were done elsewhere)
  if (getenv("YKSIM_SECONDARY")) {
    std::vector<size_t> keep;
    for (size_t i : idx)
      if (seg_depth[i] > 0) keep.push_back(i);
    idx.swap(keep);
  }
  std::shuffle(idx.begin(), idx.end(), rng);
  // YKSIM_PRIMARY=1: only the camera rays, a wave = one 8x8 pixel block at one sample (the
  // coherent first segment: how many wave-level iterations a batch of primary rays needs)
  if (getenv("YKSIM_PRIMARY")) {
    seg.clear();
    idx.clear();
    for (int by = 0; by < H; by += 8)
      for (int bx = 0; bx < W; bx += 8)
        for (int k = 0; k < 64; ++k) {
          const int x = bx + k % 8, y = by + k / 8;
          if (x >= W || y >= H) continue;
          double u = (x + U(rng)) / W, v = (H - y - 1 + U(rng)) / H;
          V o = ld(cam.origin);
          V d = sub(add(add(ld(cam.lower_left_corner), mul(ld(cam.horizontal), u)), mul(ld(cam.vertical), v)), o);
          idx.push_back(seg.size());
          seg.push_back({o, d});
        }
    // YKSIM_PRIMARY_SHUFFLE=1: the same camera rays in random waves (coherence vs ray kind)
    if (getenv("YKSIM_PRIMARY_SHUFFLE")) std::shuffle(idx.begin(), idx.end(), rng);
  }
  auto rcp = [](float x) { return std::fabs(x) > 1e-30f ? 1.0f / x : std::copysign(1e30f, x); };
  // traversal cost of one trip of the shipped (if/else) loop over an arbitrary set of rays
  auto trav_cost = [&](const std::vector<std::pair<V, V>>& rays) {
    std::vector<Lane> lanes(rays.size());
    for (size_t k = 0; k < rays.size(); ++k) {
      Lane& L = lanes[k];
      L.o = rays[k].first;
      L.d = rays[k].second;
      L.a = dot(L.d, L.d);
      L.ix = rcp((float)L.d.x), L.iy = rcp((float)L.d.y), L.iz = rcp((float)L.d.z);
      L.node = M.root;
    }
    double cost = 0;
    for (;;) {
      bool any_v = false;
      int max_cnt = 0, max_dpos = 0, act = 0;
      for (auto& L : lanes) {
        if (L.done) continue;
        ++act;
        if (L.node >= 0) {
          any_v = true;
          M.visit(L);
          if (L.node == kDone) L.done = true;
        } else {
          auto [cnt, dp] = M.leaf(L, L.node);
          max_cnt = std::max(max_cnt, cnt);
          max_dpos = std::max(max_dpos, dp);
          M.pop(L);
          if (L.node == kDone) L.done = true;
        }
      }
      if (!act) break;
      cost += c_trip + c_visit * any_v + c_leaf * max_cnt + c_disc * max_dpos;
    }
    return cost;
  };
  // YKSIM_BURST="other T Q": one wave's refill policy over the slot stream (slot order = the
  // kernel's: 8x8 pixel blocks, sample index outermost), every trip = the traversal of the active
  // lanes' current segments + `other`.  T = 0: the shipped refill (every free lane takes the next
  // slot each trip).  T > 0: park & burst — when at least T lanes are free (and the park queue,
  // FIFO of capacity Q, has room for the active ones), the active lanes are parked and the wave
  // starts 64 consecutive slots together (a coherent primary trip); otherwise free lanes take
  // parked paths, and stay idle when there are none.
  if (const char* bs = getenv("YKSIM_BURST")) {
    double other = 957, T = 0, Q = 64;
    sscanf(bs, "%lf %lf %lf", &other, &T, &Q);
    std::vector<std::vector<size_t>> path((size_t)W * H * SPP);
    {
      size_t sidx = 0;
      for (size_t i = 0; i < seg.size(); ++i) {
        if (seg_depth[i] == 0 && i > 0) ++sidx;
        path[sidx].push_back(i);
      }
    }
    std::vector<size_t> slots;  // sample index per slot
    // YKSIM_BLOCKMAJOR=1: a block's samples contiguous (block, sample, pixel) instead of
    // (sample, block, pixel)
    const bool bm = getenv("YKSIM_BLOCKMAJOR") != nullptr;
    for (int s0 = 0; s0 < (bm ? 1 : SPP); ++s0)
      for (int by = 0; by < H; by += 8)
        for (int bx = 0; bx < W; bx += 8)
          for (int s = bm ? 0 : s0; s < (bm ? SPP : s0 + 1); ++s)
            for (int k = 0; k < 64; ++k) {
              const int x = bx + k % 8, y = by + k / 8;
              if (x < W && y < H) slots.push_back(((size_t)y * W + x) * SPP + s);
            }
    struct P { size_t q; int d; };
    std::vector<P> lane(64, P{0, -1});  // d < 0: free
    std::deque<P> park;
    size_t next = 0;
    double cost = 0, trips = 0, bursts = 0, lanes_active = 0;
    for (;;) {
      int nfree = 0;
      for (auto& l : lane) nfree += l.d < 0;
      const int nact = 64 - nfree;
      if (T > 0 && nfree >= T && next < slots.size() && park.size() + nact <= Q) {
        for (auto& l : lane)
          if (l.d >= 0) park.push_back(l), l.d = -1;
        for (auto& l : lane)
          if (next < slots.size()) l = P{slots[next++], 0};
        ++bursts;
      } else {
        for (auto& l : lane) {
          if (l.d >= 0) continue;
          if (T > 0) {
            if (!park.empty()) l = park.front(), park.pop_front();
          } else if (next < slots.size()) {
            l = P{slots[next++], 0};
          }
        }
      }
      std::vector<std::pair<V, V>> rays;
      for (auto& l : lane)
        if (l.d >= 0) rays.push_back(seg[path[l.q][l.d]]);
      if (rays.empty()) {
        if (next >= slots.size() && park.empty()) break;
        if (T > 0 && next < slots.size()) {  // nothing to run: burst regardless of T
          for (auto& l : lane)
            if (next < slots.size()) l = P{slots[next++], 0};
          ++bursts;
          continue;
        }
        continue;
      }
      cost += trav_cost(rays) + other;
      trips += 1;
      lanes_active += rays.size();
      for (auto& l : lane)
        if (l.d >= 0 && ++l.d >= (int)path[l.q].size()) l.d = -1;
    }
    printf("burst(other=%.0f, T=%.0f, Q=%.0f): per sample %.1f | trips %.0f, bursts %.0f, lanes per trip %.1f\n",
           other, T, Q, cost / slots.size(), trips, bursts, lanes_active / trips);
  }
  // YKSIM_WAVESYNC=other: waves of 64 coherent samples (one 8x8 block, one sample index) traced in
  // lockstep to their end, no refill: trip d holds the samples' depth-d segments; every trip also
  // pays `other` for the rest of the loop (shading, path end, start, refill), whatever its lanes.
  // Printed beside the shipped refill loop's cost per sample (random waves of 64 segments) and
  // the split (coherent primary waves + random bounce waves)
  if (const char* ws = getenv("YKSIM_WAVESYNC")) {
    const double other = atof(ws);
    std::vector<std::vector<size_t>> path((size_t)W * H * SPP);  // segment indices per sample, (y, x, s) order
    {
      size_t sidx = 0;
      for (size_t i = 0; i < seg.size(); ++i) {
        if (seg_depth[i] == 0 && i > 0) ++sidx;
        path[sidx].push_back(i);
      }
    }
    double sync = 0, nsamp = 0, prim = 0, bounce = 0, mixed = 0, nb = 0;
    std::vector<size_t> bidx;
    for (int s = 0; s < 2; ++s)
      for (int by = 0; by < H; by += 8)
        for (int bx = 0; bx < W; bx += 8) {
          std::vector<size_t> smp;
          for (int k = 0; k < 64; ++k) {
            const int x = bx + k % 8, y = by + k / 8;
            if (x < W && y < H) smp.push_back(((size_t)y * W + x) * SPP + s);
          }
          if (smp.size() < 64) continue;
          for (int d = 0;; ++d) {
            std::vector<std::pair<V, V>> rays;
            for (size_t q : smp)
              if ((int)path[q].size() > d) rays.push_back(seg[path[q][d]]);
            if (rays.empty()) break;
            const double c = trav_cost(rays) + other;
            sync += c;
            if (d == 0) prim += c;
          }
          for (size_t q : smp)
            for (size_t k = 1; k < path[q].size(); ++k) bidx.push_back(path[q][k]);
          nsamp += smp.size();
        }
    std::shuffle(bidx.begin(), bidx.end(), rng);
    for (size_t g = 0; g + 64 <= bidx.size(); g += 64) {
      std::vector<std::pair<V, V>> rays;
      for (int k = 0; k < 64; ++k) rays.push_back(seg[bidx[g + k]]);
      bounce += trav_cost(rays) + other;
      nb += 64;
    }
    for (size_t g = 0; g + 64 <= idx.size(); g += 64) {
      std::vector<std::pair<V, V>> rays;
      for (int k = 0; k < 64; ++k) rays.push_back(seg[idx[g + k]]);
      mixed += trav_cost(rays) + other;
    }
    const double segs_per_sample = (double)seg.size() / (W * H * 2);
    const double mixed_ps = mixed / (idx.size() / 64) / 64 * segs_per_sample;
    const double split_ps = prim / nsamp + bounce / nb * (bidx.size() / nsamp);
    printf("wavesync(other=%.0f): per sample: refill loop (random waves) %.1f | lockstep coherent waves %.1f (%.3fx) | "
           "coherent primary waves + random bounce waves %.1f (%.3fx)\n",
           other, mixed_ps, sync / nsamp, sync / nsamp / mixed_ps, split_ps, split_ps / mixed_ps);
  }

  printf("%s n=%u leaf<=%u wide nodes %zu depth %u | %zu segments | weights visit %.0f leaf %.0f disc %.0f trip %.0f\n",
         scene, n, opt.max_leaf, M.wide.size(), wd, seg.size(), c_visit, c_leaf, c_disc, c_trip);
  if (const char* we = getenv("YKSIM_WIDTH")) {
    const int width = atoi(we);
    std::vector<WideN> wn;
    collapse_n(b, wn, b.root, width);
    double vb = 0, lb = 0, lv = 0, ll = 0;
    size_t nw = 0;
    for (size_t g = 0; g + 64 <= idx.size(); g += 64, ++nw) {
      struct L { V o, d; double a, ustar = INFINITY; float ix, iy, iz, uf = INFINITY; std::vector<int32_t> st; int32_t node = 0; bool done = false; };
      std::vector<L> ls(64);
      for (int k = 0; k < 64; ++k) {
        L& x = ls[k];
        x.o = seg[idx[g + k]].first; x.d = seg[idx[g + k]].second; x.a = dot(x.d, x.d);
        x.ix = rcp((float)x.d.x); x.iy = rcp((float)x.d.y); x.iz = rcp((float)x.d.z);
      }
      for (;;) {
        bool av = false, al = false, act = false;
        for (auto& x : ls) {
          if (x.done) continue;
          act = true;
          if (x.node >= 0) {
            av = true; ++lv;
            const WideN& w = wn[x.node];
            int last = -1;
            bool hk[8];
            for (int k = 0; k < w.n; ++k) {
              const float i3[3] = {x.ix, x.iy, x.iz};
              const double o3[3] = {x.o.x, x.o.y, x.o.z};
              float tn = 0.001f, tf = x.uf;
              for (int a = 0; a < 3; ++a) {
                float t0 = (w.lo[k][a] - (float)o3[a]) * i3[a], t1 = (w.hi[k][a] - (float)o3[a]) * i3[a];
                tn = std::max(tn, std::min(t0, t1)); tf = std::min(tf, std::max(t0, t1));
              }
              hk[k] = tn <= tf * (1 + 0x1p-17f);
              if (hk[k]) last = k;
            }
            if (last < 0) {
              if (x.st.empty()) x.done = true; else { x.node = x.st.back(); x.st.pop_back(); }
            } else {
              for (int k = 0; k < last; ++k) if (hk[k]) x.st.push_back(w.code[k]);
              x.node = w.code[last];
            }
          } else {
            al = true;
            Lane tmp; tmp.o = x.o; tmp.d = x.d; tmp.a = x.a; tmp.ustar = x.ustar; tmp.uf = x.uf;
            auto [cnt, dp] = M.leaf(tmp, x.node);
            (void)dp; ll += cnt;
            x.ustar = tmp.ustar; x.uf = tmp.uf;
            if (x.st.empty()) x.done = true; else { x.node = x.st.back(); x.st.pop_back(); }
          }
        }
        if (!act) break;
        vb += av; lb += al;
      }
    }
    printf("width %d: %zu nodes | per wave-segment: visit blocks %.1f, leaf blocks %.1f | per lane: visits %.2f, leaf tests %.2f\n",
           width, wn.size(), vb / nw, lb / nw, lv / (64.0 * nw), ll / (64.0 * nw));
  }
  // ---- wave work-pool models: one LIFO of (ray, node) pairs per wave, 64 pairs per trip
  // pool 0: nodes and leaves mixed in the pool; pool 1: leaves go to a list tested 64 at a time
  // (when it holds 64, or the node pool is empty)
  for (int pv = 0; pv < 2; ++pv) {
    double trips = 0, vis_trips = 0, leaf_trips = 0, lv = 0, ll = 0, cost = 0, maxpool = 0, ovf = 0, cand = 0;
    std::vector<size_t> ins_hist(16, 0);
    size_t nw = 0;
    for (size_t g = 0; g + 64 <= idx.size(); g += 64, ++nw) {
      std::vector<Lane> lanes(64);
      std::vector<std::pair<int, int32_t>> pool, leaves;
      std::vector<int> ncand(64, 0);
      std::vector<std::vector<float>> lbs(64);
      for (int k = 0; k < 64; ++k) {
        Lane& L = lanes[k];
        L.o = seg[idx[g + k]].first;
        L.d = seg[idx[g + k]].second;
        L.a = dot(L.d, L.d);
        L.ix = rcp((float)L.d.x), L.iy = rcp((float)L.d.y), L.iz = rcp((float)L.d.z);
        pool.push_back({k, M.root});
      }
      auto leaf_test = [&](int k, int32_t code) {
        Lane& L = lanes[k];
        const uint32_t v = ~(uint32_t)code, first = v >> 4, cnt = v & 15u;
        for (uint32_t q = 0; q < cnt; ++q) {
          const yk_sphere& s = M.sph[M.order[first + q]];
          V oc = sub(L.o, ld(s.center));
          double hb = dot(oc, L.d), cc = dot(oc, oc) - s.radius * s.radius;
          double disc = hb * hb - L.a * cc;
          ++ll;
          if (disc < 0) continue;
          double sq = std::sqrt(disc), r1 = (-hb - sq) / L.a, r2 = (-hb + sq) / L.a;
          double lb = r1 >= 0.001 ? r1 : r2;
          double ub = r1 >= 0.001 ? r1 : (r2 >= 0.001 ? r2 : INFINITY);
          if (!(lb <= L.ustar)) continue;
          if (ub < L.ustar) { L.ustar = ub; L.uf = (float)ub * (1 + 0x1p-18f); }
          lbs[k].push_back((float)lb);
        }
      };
      while (!pool.empty() || !leaves.empty()) {
        std::vector<std::pair<int, int32_t>> take;
        bool leaf_trip = false;
        if (pv == 1 && (leaves.size() >= 64 || pool.empty())) {
          const size_t n = std::min<size_t>(64, leaves.size());
          take.assign(leaves.end() - n, leaves.end());
          leaves.resize(leaves.size() - n);
          leaf_trip = true;
        } else {
          const size_t n = std::min<size_t>(64, pool.size());
          take.assign(pool.end() - n, pool.end());
          pool.resize(pool.size() - n);
        }
        // snapshot of U* at the trip's start (updates land after the trip)
        std::vector<float> uf(64);
        for (int k = 0; k < 64; ++k) uf[k] = lanes[k].uf;
        bool any_v = false, any_l = false;
        std::vector<std::pair<int, int32_t>> pushed;
        for (auto [k, code] : take) {
          if (code >= 0) {
            any_v = true;
            ++lv;
            Lane L = lanes[k];
            L.uf = uf[k];
            L.stk.clear();
            L.node = code;
            M.visit(L);
            // children entered: the stack (in push order) plus the next node
            for (int32_t c : L.stk) pushed.push_back({k, c});
            if (L.node != kDone) pushed.push_back({k, L.node});
          } else if (code != ykbvh::kEmptyLeaf) {
            any_l = true;
            leaf_test(k, code);
          }
        }
        for (auto& e : pushed) {
          if (pv == 1 && e.second < 0) leaves.push_back(e);
          else pool.push_back(e);
        }
        maxpool = std::max(maxpool, (double)(pool.size() + leaves.size()));
        trips += 1;
        vis_trips += any_v;
        leaf_trips += any_l;
        cost += c_trip + (any_v ? c_visit + 25 : 0) + (any_l ? c_leaf + c_disc + 25 : 0);
      }
      for (int k = 0; k < 64; ++k) {
        int n = 0;
        for (float lb : lbs[k]) n += lb <= lanes[k].uf;
        cand += n;
        ovf += lbs[k].size() > 4;
        ins_hist[std::min<size_t>(lbs[k].size(), 15)]++;
      }
    }
    printf("pool %d: per wave-segment: trips %.1f (visit %.1f, leaf %.1f) | per lane: visits %.2f leaf tests %.2f, "
           "final candidates %.2f, inserted > 4: %.5f | max pool %.0f | cost %.0f\n",
           pv, trips / nw, vis_trips / nw, leaf_trips / nw, lv / (64.0 * nw), ll / (64.0 * nw), cand / (64.0 * nw),
           ovf / (64.0 * nw), maxpool, cost / nw);
    printf("  inserted candidates per ray:");
    for (int q = 0; q < 16; ++q) printf(" [%d]%zu", q, ins_hist[q]);
    printf("\n");
  }
  // ---- round 4: two traversals per lane (rays k and k + 64 of a 128-ray wave, each the ifelse
  // loop; one trip issues both rays' blocks) and a two-node frontier of ONE ray per lane (the
  // current node and, when it is an inner node, the stack top's inner node visited in the same
  // trip; the last entered child of the pair is next, the rest pushed)
  {
    double trips = 0, vb = 0, lb = 0, lv = 0, ll = 0, rounds = 0;
    size_t nw = 0;
    std::vector<size_t> sthist(20, 0);
    for (size_t g = 0; g + 128 <= idx.size(); g += 128, ++nw) {
      std::vector<Lane> lanes(128);
      for (int k = 0; k < 128; ++k) {
        Lane& L = lanes[k];
        L.o = seg[idx[g + k]].first;
        L.d = seg[idx[g + k]].second;
        L.a = dot(L.d, L.d);
        L.ix = rcp((float)L.d.x), L.iy = rcp((float)L.d.y), L.iz = rcp((float)L.d.z);
        L.node = M.root;
      }
      for (;;) {
        bool act = false, v[2] = {false, false}, l[2] = {false, false};
        for (int k = 0; k < 128; ++k) {
          Lane& L = lanes[k];
          if (L.done) continue;
          act = true;
          if (L.node >= 0) {
            v[k >> 6] = true, ++lv;
            M.visit(L);
            if (L.node == kDone) L.done = true;
          } else {
            l[k >> 6] = true;
            ll += M.leaf(L, L.node).first;
            M.pop(L);
            if (L.node == kDone) L.done = true;
          }
        }
        for (auto& L : lanes) L.pend = std::max<int32_t>(L.pend, (int32_t)L.stk.size());
        if (!act) break;
        trips += 1;
        vb += v[0] + v[1];
        lb += l[0] + l[1];
      }
      for (auto& L : lanes) sthist[std::min<int32_t>(L.pend, 19)]++;
    }
    printf("stack depth (max per ray):");
    for (int q = 0; q < 20; ++q) if (sthist[q]) printf(" [%d]%zu", q, sthist[q]);
    printf("\n");
    printf("2 rays/lane (128/wave)  per wave-trip-of-2-segments: trips %.1f, visit blocks %.1f, leaf blocks %.1f | "
           "per ray: visits %.2f leaf tests %.2f\n",
           trips / nw, vb / nw, lb / nw, lv / (128.0 * nw), ll / (128.0 * nw));
    (void)rounds;
  }
  {
    double trips = 0, vb = 0, vb2 = 0, lb = 0, lv = 0, ll = 0;
    size_t nw = 0, maxst = 0;
    for (size_t g = 0; g + 64 <= idx.size(); g += 64, ++nw) {
      std::vector<Lane> lanes(64);
      for (int k = 0; k < 64; ++k) {
        Lane& L = lanes[k];
        L.o = seg[idx[g + k]].first;
        L.d = seg[idx[g + k]].second;
        L.a = dot(L.d, L.d);
        L.ix = rcp((float)L.d.x), L.iy = rcp((float)L.d.y), L.iz = rcp((float)L.d.z);
        L.node = M.root;
      }
      for (;;) {
        bool act = false, v = false, v2 = false, l = false;
        for (auto& L : lanes) {
          if (L.done) continue;
          act = true;
          if (L.node >= 0) {
            v = true, ++lv;
            int32_t second = kDone;
            if (!L.stk.empty() && L.stk.back() >= 0) {
              second = L.stk.back();
              L.stk.pop_back();
            }
            // visit the first: its entered children (stack pushes + next)
            Lane A = L;
            A.stk.clear();
            M.visit(A);  // A.node: next or kDone (after an empty pop of an empty stack)
            std::vector<int32_t> ch(A.stk);
            if (A.node != kDone) ch.push_back(A.node);
            if (second != kDone) {
              v2 = true, ++lv;
              Lane B = L;
              B.stk.clear();
              B.node = second;
              M.visit(B);
              for (int32_t c2 : B.stk) ch.push_back(c2);
              if (B.node != kDone) ch.push_back(B.node);
            }
            if (ch.empty()) {
              M.pop(L);
            } else {
              L.node = ch.back();
              ch.pop_back();
              for (int32_t c2 : ch) L.stk.push_back(c2);
            }
            maxst = std::max(maxst, L.stk.size());
            if (L.node == kDone) L.done = true;
          } else {
            l = true;
            ll += M.leaf(L, L.node).first;
            M.pop(L);
            if (L.node == kDone) L.done = true;
          }
        }
        if (!act) break;
        trips += 1;
        vb += v;
        vb2 += v2;
        lb += l;
      }
    }
    printf("frontier-2              per wave-segment: trips %.1f, visit blocks %.1f (second visits %.1f), leaf blocks %.1f | "
           "per lane: visits %.2f leaf tests %.2f | max stack %zu\n",
           trips / nw, vb / nw, vb2 / nw, lb / nw, lv / (64.0 * nw), ll / (64.0 * nw), maxst);
  }
  for (int variant = 0; variant < 4; ++variant) {
    double trips = 0, wv = 0, wl = 0, wd2 = 0, lv = 0, ll = 0, cost = 0;
    size_t nw = 0;
    for (size_t g = 0; g + 64 <= idx.size(); g += 64, ++nw) {
      std::vector<Lane> lanes(64);
      for (int k = 0; k < 64; ++k) {
        Lane& L = lanes[k];
        L.o = seg[idx[g + k]].first;
        L.d = seg[idx[g + k]].second;
        L.a = dot(L.d, L.d);
        L.ix = rcp((float)L.d.x), L.iy = rcp((float)L.d.y), L.iz = rcp((float)L.d.z);
        L.node = M.root;
      }
      for (;;) {
        bool any_v = false, any_l = false;
        int max_cnt = 0, max_dpos = 0, act = 0;
        // variant 3 (Aila-Laine speculative): leaves are tested only when every active lane has
        // one parked or nothing left to visit
        bool test_now = true;
        if (variant == 3) {
          int ready = 0, live = 0;
          for (auto& L : lanes)
            if (!L.done) {
              ++live;
              ready += !(L.pend == kNone && L.node != kDone);
            }
          test_now = ready >= frac * live;
        }
        for (auto& L : lanes) {
          if (L.done) continue;
          ++act;
          if (variant == 3) {
            if (test_now && L.pend != kNone) {
              any_l = true;
              auto [cnt, dp] = M.leaf(L, L.pend);
              ll += cnt;
              max_cnt = std::max(max_cnt, cnt);
              max_dpos = std::max(max_dpos, dp);
              L.pend = kNone;
            }
            if (L.node >= 0) {
              any_v = true;
              ++lv;
              M.visit(L);
            }
            if (L.pend == kNone && L.node != kDone && L.node < 0) {
              L.pend = L.node;
              M.pop(L);
            }
            if (L.node == kDone && L.pend == kNone) L.done = true;
          } else if (variant == 0) {  // ifelse
            if (L.node >= 0) {
              any_v = true;
              ++lv;
              M.visit(L);
              if (L.node == kDone) L.done = true;
            } else {
              any_l = true;
              auto [cnt, dp] = M.leaf(L, L.node);
              ll += cnt;
              max_cnt = std::max(max_cnt, cnt);
              max_dpos = std::max(max_dpos, dp);
              M.pop(L);
              if (L.node == kDone) L.done = true;
            }
          } else {  // postpone (variant 2: the leaf test before the visit)
            auto do_leaf = [&]() {
              if (L.pend != kNone) {
                any_l = true;
                auto [cnt, dp] = M.leaf(L, L.pend);
                ll += cnt;
                max_cnt = std::max(max_cnt, cnt);
                max_dpos = std::max(max_dpos, dp);
                L.pend = kNone;
              }
            };
            if (variant == 2) do_leaf();
            if (L.node >= 0) {
              any_v = true;
              ++lv;
              M.visit(L);
            }
            if (L.pend == kNone && L.node != kDone && L.node < 0) {
              L.pend = L.node;
              M.pop(L);
            }
            if (variant == 1) do_leaf();
            if (L.node == kDone && L.pend == kNone) L.done = true;
          }
        }
        if (!act) break;
        trips += 1;
        wv += any_v;
        wl += max_cnt;
        wd2 += max_dpos;
        cost += c_trip + c_visit * any_v + c_leaf * max_cnt + c_disc * max_dpos;
      }
    }
    const char* name[4] = {"ifelse", "postpone(visit,leaf)", "postpone(leaf,visit)", "speculative"};
    printf("%-22s per wave-segment: trips %.1f, visit blocks %.1f, leaf iters %.1f, disc tails %.1f | "
           "per lane: visits %.2f leaf tests %.2f | cost %.0f\n",
           name[variant], trips / nw, wv / nw, wl / nw, wd2 / nw, lv / (64.0 * nw), ll / (64.0 * nw), cost / nw);
  }
  // ---- round 6: the branch-free visit's while-while loop (YK_NODE_BF: an inner visit loop until
  // every lane holds a leaf, then one leaf block, then the pops) and its speculative form (a visit
  // whose last entered child is a leaf parks it and goes on with the entry below the new top, known
  // in registers; the leaf block tests the parked leaf, else the lane's current leaf)
  for (int spec = 0; spec < 2; ++spec) {
    double vb = 0, lb = 0, db = 0, outer = 0, lv = 0, ll = 0;
    size_t nw = 0;
    for (size_t g = 0; g + 64 <= idx.size(); g += 64, ++nw) {
      std::vector<Lane> lanes(64);
      for (int k = 0; k < 64; ++k) {
        Lane& L = lanes[k];
        L.o = seg[idx[g + k]].first;
        L.d = seg[idx[g + k]].second;
        L.a = dot(L.d, L.d);
        L.ix = rcp((float)L.d.x), L.iy = rcp((float)L.d.y), L.iz = rcp((float)L.d.z);
        L.node = M.root;
      }
      for (;;) {
        outer += 1;
        for (;;) {  // inner: visits
          bool any = false;
          for (auto& L : lanes) {
            if (L.done || L.node < 0) continue;
            any = true;
            ++lv;
            const size_t before = L.stk.size();
            M.visit(L);
            const bool entered = !(L.stk.size() + 1 == before || (before == 0 && L.node == kDone && false));
            // a pop inside the visit shrinks the stack by one; anything else entered a slot
            const bool popped = L.stk.size() + 1 == before && L.node != kDone;
            if (spec && !popped && entered && L.node < 0 && L.node != kDone && L.pend == kNone) {
              L.pend = L.node;
              M.pop(L);
            }
          }
          if (!any) break;
          vb += 1;
        }
        bool anyl = false;
        int maxd = 0;
        for (auto& L : lanes) {
          if (L.done) continue;
          int32_t leaf = kNone;
          if (L.pend != kNone) {
            leaf = L.pend;
            L.pend = kNone;
          } else if (L.node < 0 && L.node != kDone) {
            leaf = L.node;
            M.pop(L);
          }
          if (leaf != kNone) {
            anyl = true;
            auto [cnt, dp] = M.leaf(L, leaf);
            ll += cnt;
            maxd = std::max(maxd, dp);
          }
          // a lane still holding a leaf parks it (spec) or keeps it for the next block
          if (spec && L.node < 0 && L.node != kDone && L.pend == kNone) {
            L.pend = L.node;
            M.pop(L);
          }
          if (L.node == kDone && L.pend == kNone) L.done = true;
        }
        lb += anyl;
        db += maxd;
        bool all = true;
        for (auto& L : lanes) all = all && L.done;
        if (all) break;
      }
    }
    printf("%-22s per wave-segment: outer %.1f, visit blocks %.1f, leaf blocks %.1f, disc tails %.1f | per lane: visits %.2f leaf tests %.2f | cost %.0f\n",
           spec ? "BF speculative" : "BF while-while", outer / nw, vb / nw, lb / nw, db / nw, lv / (64.0 * nw), ll / (64.0 * nw),
           (c_trip * outer + c_visit * vb + c_leaf * lb + c_disc * db) / nw);
  }
  return 0;
}
