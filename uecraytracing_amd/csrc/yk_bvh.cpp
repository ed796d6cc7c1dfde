// yk_bvh.cpp — binned-SAH BVH builder (host).  See yk_bvh.hpp for the culling contract.
#include "yk_bvh.hpp"

#include <algorithm>
#include <cmath>
#include <numeric>

namespace ykbvh {
namespace {

struct Box {
  double lo[3] = {INFINITY, INFINITY, INFINITY};
  double hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const Box& b) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], b.lo[k]);
      hi[k] = std::max(hi[k], b.hi[k]);
    }
  }
  void grow(const double* p) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], p[k]);
      hi[k] = std::max(hi[k], p[k]);
    }
  }
  double area() const {
    if (!(hi[0] >= lo[0])) return 0;
    const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return 2 * (dx * dy + dy * dz + dz * dx);
  }
};

struct Builder {
  const double* c;
  std::vector<Box> sbox;     // per sphere, grown by delta
  std::vector<double> cent;  // centroids
  std::vector<uint32_t> idx;
  std::vector<Node> nodes;
  bool median_only = false;
  uint32_t max_depth = 0;
  Options opt;

  Box bounds(uint32_t b, uint32_t e) const {
    Box r;
    for (uint32_t i = b; i < e; ++i) r.grow(sbox[idx[i]]);
    return r;
  }

  // returns a child code for the subtree over idx[b, e)
  int32_t rec(uint32_t b, uint32_t e, uint32_t depth) {
    const uint32_t n = e - b;
    if (n <= opt.max_leaf) {
      max_depth = std::max(max_depth, depth);
      return ~int32_t((b << 4) | n);
    }
    Box cb;
    for (uint32_t i = b; i < e; ++i) cb.grow(&cent[3 * idx[i]]);
    int axis = 0;
    for (int k = 1; k < 3; ++k)
      if (cb.hi[k] - cb.lo[k] > cb.hi[axis] - cb.lo[axis]) axis = k;
    uint32_t mid = b + n / 2;
    double ext = cb.hi[axis] - cb.lo[axis];
    if (!median_only && ext > 0) {
      const int kBins = std::min(std::max(opt.bins, 2), 256);
      // binned SAH over the longest centroid axis, or (opt.all_axes) the cheapest of the three
      double best = INFINITY;
      int best_q = -1, best_axis = axis;
      for (int ax = 0; ax < 3; ++ax) {
        if (!opt.all_axes && ax != axis) continue;
        const double ex = cb.hi[ax] - cb.lo[ax];
        if (!(ex > 0)) continue;
        std::vector<Box> bb(kBins);
        std::vector<uint32_t> cnt(kBins, 0);
        for (uint32_t i = b; i < e; ++i) {
          const uint32_t sp = idx[i];
          const int q = std::min(std::max(int((cent[3 * sp + ax] - cb.lo[ax]) / ex * kBins), 0), kBins - 1);
          bb[q].grow(sbox[sp]);
          ++cnt[q];
        }
        for (int q = 1; q < kBins; ++q) {
          Box l, r;
          uint32_t nl = 0, nr = 0;
          for (int t = 0; t < q; ++t) { l.grow(bb[t]); nl += cnt[t]; }
          for (int t = q; t < kBins; ++t) { r.grow(bb[t]); nr += cnt[t]; }
          if (!nl || !nr) continue;
          const double cost = l.area() * nl + r.area() * nr;
          if (cost < best) { best = cost; best_q = q; best_axis = ax; }
        }
      }
      axis = best_axis;
      ext = cb.hi[axis] - cb.lo[axis];
      auto bin_of = [&](uint32_t sp) {
        int q = int((cent[3 * sp + axis] - cb.lo[axis]) / ext * kBins);
        return std::min(std::max(q, 0), kBins - 1);
      };
      if (best_q > 0) {
        auto it = std::partition(idx.begin() + b, idx.begin() + e,
                                 [&](uint32_t sp) { return bin_of(sp) < best_q; });
        mid = uint32_t(it - idx.begin());
      }
    }
    if (mid == b || mid == e || median_only || ext == 0) {
      mid = b + n / 2;
      std::nth_element(idx.begin() + b, idx.begin() + mid, idx.begin() + e,
                       [&](uint32_t x, uint32_t y) { return cent[3 * x + axis] < cent[3 * y + axis]; });
    }
    const int32_t me = int32_t(nodes.size());
    nodes.emplace_back();
    const int32_t l = rec(b, mid, depth + 1);
    const int32_t r = rec(mid, e, depth + 1);
    const Box bl = bounds(b, mid), br = bounds(mid, e);
    Node& nd = nodes[me];
    const Box* kids[2] = {&bl, &br};
    for (int k = 0; k < 2; ++k) {
      // outward rounding to float: nextafter past the double bound
      auto dn = [](double v) { float f = (float)v; return (double)f > v ? std::nextafter(f, -INFINITY) : f; };
      auto up = [](double v) { float f = (float)v; return (double)f < v ? std::nextafter(f, INFINITY) : f; };
      nd.lo_x[k] = dn(kids[k]->lo[0]);
      nd.lo_y[k] = dn(kids[k]->lo[1]);
      nd.lo_z[k] = dn(kids[k]->lo[2]);
      nd.hi_x[k] = up(kids[k]->hi[0]);
      nd.hi_y[k] = up(kids[k]->hi[1]);
      nd.hi_z[k] = up(kids[k]->hi[2]);
    }
    nd.child[0] = l;
    nd.child[1] = r;
    nd.pad[0] = nd.pad[1] = 0;
    return me;
  }
};

}  // namespace

Built build(const double* centers, const double* radii, uint32_t n, double camera_extent,
            const Options& opt) {
  Built out;
  double ext = camera_extent;
  for (uint32_t i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) ext = std::max(ext, std::fabs(centers[3 * i + k]) + std::fabs(radii[i]));
  // origins of secondary rays lie on sphere surfaces (|o| <= ext); allow 4x headroom
  out.origin_bound = 4.0 * ext;
  out.delta = (float)std::ldexp(out.origin_bound, -21);
  for (int attempt = 0; attempt < 2; ++attempt) {
    Builder bd;
    bd.c = centers;
    bd.median_only = attempt == 1;
    bd.opt = opt;
    bd.sbox.resize(n);
    bd.cent.assign(centers, centers + 3 * size_t(n));
    bd.idx.resize(n);
    std::iota(bd.idx.begin(), bd.idx.end(), 0u);
    for (uint32_t i = 0; i < n; ++i) {
      const double ar = std::fabs(radii[i]);
      double g = ar * opt.radius_grow;
      if (opt.f32_big) {
        const double* c = centers + 3 * i;
        const double reach = std::sqrt(3.0) * out.origin_bound + std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]) + ar;
        if (kF32BigReach * ar >= reach * (1.0 + 0x1p-20)) g = std::min(g, ar * kF32BigGrow);
      }
      const double r = ar + g + out.delta;
      for (int k = 0; k < 3; ++k) {
        bd.sbox[i].lo[k] = centers[3 * i + k] - r;
        bd.sbox[i].hi[k] = centers[3 * i + k] + r;
      }
    }
    out.root = bd.rec(0, n, 0);
    out.depth = bd.max_depth;
    if (out.depth <= kMaxDepth || attempt == 1) {
      out.nodes = std::move(bd.nodes);
      out.order = std::move(bd.idx);
      break;
    }
  }
  return out;
}


namespace {
struct Slot {
  float lo[3], hi[3];
  int32_t code;  // binary-tree code: >= 0 inner node index, < 0 leaf
};

float slot_area(const Slot& e) {
  const float dx = e.hi[0] - e.lo[0], dy = e.hi[1] - e.lo[1], dz = e.hi[2] - e.lo[2];
  return dx * dy + dy * dz + dz * dx;
}

Slot child_slot(const Node& n, int k) {
  return Slot{{n.lo_x[k], n.lo_y[k], n.lo_z[k]}, {n.hi_x[k], n.hi_y[k], n.hi_z[k]}, n.child[k]};
}

// Emits the wide node for binary inner node `idx` (and its subtree) into out; returns its index.
uint32_t collapse(const Built& b, int32_t idx, std::vector<WideNode>& out, uint32_t depth, uint32_t& max_depth) {
  std::vector<Slot> slots = {child_slot(b.nodes[idx], 0), child_slot(b.nodes[idx], 1)};
  while (slots.size() < 4) {
    int best = -1;
    for (size_t i = 0; i < slots.size(); ++i)
      if (slots[i].code >= 0 && (best < 0 || slot_area(slots[i]) > slot_area(slots[best]))) best = (int)i;
    if (best < 0) break;
    const Node& c = b.nodes[slots[best].code];
    slots[best] = child_slot(c, 0);
    slots.insert(slots.begin() + best + 1, child_slot(c, 1));  // siblings stay adjacent
  }
  max_depth = std::max(max_depth, depth + 1);
  const uint32_t me = (uint32_t)out.size();
  out.emplace_back();
  int32_t codes[4];
  for (int k = 0; k < 4; ++k) {
    if (k >= (int)slots.size()) {
      codes[k] = kEmptyLeaf;
    } else if (slots[k].code >= 0) {
      codes[k] = (int32_t)(collapse(b, slots[k].code, out, depth + 1, max_depth) * sizeof(WideNode));
    } else {
      codes[k] = slots[k].code;
    }
  }
  WideNode& w = out[me];
  float* ax[3] = {w.x, w.y, w.z};
  for (int k = 0; k < 4; ++k) {
    const bool used = k < (int)slots.size();
    for (int a = 0; a < 3; ++a) {
      const float lo = used ? slots[k].lo[a] : 3e38f, hi = used ? slots[k].hi[a] : -3e38f;
      ax[a][k] = lo;
      ax[a][4 + k] = hi;
      ax[a][8 + k] = lo;
    }
    w.child[k] = codes[k];
  }
  return me;
}
}  // namespace

std::vector<WideNode> wide_nodes(const Built& b, int32_t* root_code, uint32_t* wide_depth) {
  std::vector<WideNode> out;
  uint32_t depth = 0;
  if (b.root >= 0) {
    collapse(b, b.root, out, 0, depth);
    *root_code = 0;
  } else {
    *root_code = b.root;  // a single leaf
  }
  *wide_depth = depth;
  return out;
}

}  // namespace ykbvh
