// yk_dual.hpp — the FP64 mt19937 render kernel with TWO paths per lane (included by
// ykgpu_render.hip inside its anonymous namespace, after yk_render_persistent).
//
// yk_render_persistent runs one path per lane at three 768-thread render waves per SIMD, and its
// node loop is bound by the LDS round trip of each visit, not by issue: a
// wave-level node iteration takes ~1100 wave-cycles for ~57 VALU instructions.  Here every lane
// owns two independent paths (A and B) and the traversal loop visits one node of EACH per trip:
// both rays' plane reads are issued before either is waited for, so one LDS round trip serves two
// visits.  512-thread workgroups (two render waves per SIMD, 1024 paths per CU) keep the render's
// registers at <= 192 so that the yk_mt_warmup waves still fit beside it.  (tools/loopsim.cpp,
// "2 rays/lane": 18.3 wave trips per 128 ray segments against 2 x 16.4 for two 64-ray waves, with
// the same visit and leaf blocks issued.)
//
// Every path's arithmetic, draw order and result are yk_render_persistent's operation for
// operation (the phases are the same code, applied to A and then to B); only the interleaving of
// two paths' traversals in one loop is new, and the closest-hit result does not depend on visit
// order.
#pragma once

#ifndef YK_DUAL_BLOCK
#define YK_DUAL_BLOCK 512
#endif
constexpr int kDualBlock = YK_DUAL_BLOCK;
constexpr int kDualRays = 2 * kDualBlock;  // paths per workgroup (traversal stacks per workgroup)
constexpr int32_t kTravDone = INT32_MIN;   // this ray's traversal has ended (not a leaf code in use)

template <class Gen>
struct DPath {
  uint32_t slot, depth, nstk;
  uint32_t st0, st1, st2, st3;  // attenuation ids, newest in st0's low half
  v3 o, d;
  bool in_path, live;  // live: the launch may still give this path slot a sample
  Gen g;
  uint16_t* id_spill;
};

// One ray's traversal state (yk_render_persistent's locals of the BVH branch, in fewer registers:
// the slab constants of an axis as ONE register pair (1/d, -o/d) read by op_sel (dual_slab), the
// upper bound only as its float ustar_f, the candidates' tuple indices two per register)
struct DTrav {
  f2 sx, sy, sz;  // near: plane * (1/d) - o * (1/d), as (1/d, -o (1/d))
  f2 fx, fy, fz;  // far, scaled by c = 1 + 2^-17: (c/d, -o (c/d))
  const char* px;
  const char* py;
  const char* pz;
  double a, ia;
  float ustar_f;  // >= U* (1 + 2^-18): U*, the least proven upper bound of the minimum root
  uint32_t nc, c01, c23;  // candidate tuple indices (< 65536), entry k in bits 16 (k & 1) of c01 / c23
  float l0, l1, l2, l3;
  int32_t node;
  int32_t* top;
  bool linear;
};

__device__ __forceinline__ uint32_t dual_cand(const DTrav& T, int k) {
  const uint32_t w = k < 2 ? T.c01 : T.c23;
  return (k & 1) ? (w >> 16) : (w & 0xffffu);
}

// The BVH set-up of one ray (yk_render_persistent: `if (alive) { ... if (!linear) {`).
__device__ __forceinline__ void dual_trav_setup(DTrav& T, const KernelArgs& ka, const char* nodes, bool alive,
                                                v3 o, v3 d, int32_t* stk) {
  T.node = kTravDone;
  T.top = stk;
  T.nc = 0;
  T.c01 = T.c23 = 0;
  T.l0 = T.l1 = T.l2 = T.l3 = 0.0f;
  T.ustar_f = INFINITY;
  T.linear = false;
  T.a = 0.0;
  T.ia = 0.0;
  if (!alive) return;
  T.a = ykd::len2(d);
  const double onorm = fmax(fabs(o.x), fmax(fabs(o.y), fabs(o.z)));
  T.linear = (ka.flags & kFlagLinearScan) || !(T.a > 0 && T.a < INFINITY) || !(onorm <= ka.origin_bound);
  if (T.linear) return;
  const float dxf = (float)d.x, dyf = (float)d.y, dzf = (float)d.z;
  const float dmin = fminf(fminf(fabsf(dxf), fabsf(dyf)), fabsf(dzf));
  const float dmax = fmaxf(fmaxf(fabsf(dxf), fabsf(dyf)), fabsf(dzf));
  float ix, iy, iz;
  if (__ballot(!(dmin > 1e-30f && dmax < 1e30f)) == 0) {
    ix = __builtin_amdgcn_rcpf(dxf);
    iy = __builtin_amdgcn_rcpf(dyf);
    iz = __builtin_amdgcn_rcpf(dzf);
  } else {
    ix = safe_rcp(dxf);
    iy = safe_rcp(dyf);
    iz = safe_rcp(dzf);
  }
  const float oix = (float)o.x * ix, oiy = (float)o.y * iy, oiz = (float)o.z * iz;
  T.px = nodes + (ix < 0.0f ? 16u : 0u);
  T.py = nodes + 48u + (iy < 0.0f ? 16u : 0u);
  T.pz = nodes + 96u + (iz < 0.0f ? 16u : 0u);
  constexpr float kFar = 1.0f + 0x1p-17f;
  T.sx = f2{ix, -oix}, T.sy = f2{iy, -oiy}, T.sz = f2{iz, -oiz};
  const float ixs = ix * kFar, iys = iy * kFar, izs = iz * kFar;
  const float ox_f = (float)o.x, oy_f = (float)o.y, oz_f = (float)o.z;
  T.fx = f2{ixs, -(ox_f * ixs)}, T.fy = f2{iys, -(oy_f * iys)}, T.fz = f2{izs, -(oz_f * izs)};
  T.ia = ykd::rcp_bound(T.a);
  T.node = ka.bvh_root;
}

// The slab test of one wide node (yk_render_persistent's visit, the same arithmetic)
__device__ __forceinline__ uint32_t dual_slots(const DTrav& T, float tmin_lo, f4 qnx, f4 qfx, f4 qny, f4 qfy, f4 qnz,
                                               f4 qfz) {
  const f2 nx[2] = {slab_fma(qnx.xy, T.sx), slab_fma(qnx.zw, T.sx)};
  const f2 fx[2] = {slab_fma(qfx.xy, T.fx), slab_fma(qfx.zw, T.fx)};
  const f2 ny[2] = {slab_fma(qny.xy, T.sy), slab_fma(qny.zw, T.sy)};
  const f2 fy[2] = {slab_fma(qfy.xy, T.fy), slab_fma(qfy.zw, T.fy)};
  const f2 nz[2] = {slab_fma(qnz.xy, T.sz), slab_fma(qnz.zw, T.sz)};
  const f2 fz[2] = {slab_fma(qfz.xy, T.fz), slab_fma(qfz.zw, T.fz)};
  uint32_t hit = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float tn = slab_max(slab_max3(nx[k >> 1][k & 1], ny[k >> 1][k & 1], nz[k >> 1][k & 1]), tmin_lo);
    const float tf = slab_min(slab_min3(fx[k >> 1][k & 1], fy[k >> 1][k & 1], fz[k >> 1][k & 1]), T.ustar_f);
    hit |= (tn <= tf) ? (1u << k) : 0u;
  }
  return hit;
}

// After a visit: the last slot entered is next, the others entered are pushed in slot order (each
// write lands at the current top, which moves only for a push); no slot entered: pop (an empty
// stack ends the traversal).  yk_render_persistent's push/pop, with the done code for an empty pop.
__device__ __forceinline__ void dual_advance(DTrav& T, uint32_t hk, int4 ch, int32_t* stk, int32_t* stk_cap,
                                             uint32_t stack_cap) {
  const bool h0 = hk & 1u, h1 = hk & 2u, h2 = hk & 4u, h3 = hk & 8u;
  if (hk != 0) {
    T.node = h3 ? ch.w : (h2 ? ch.z : (h1 ? ch.y : ch.x));
    int32_t* top = T.top;
    *top = ch.x;
    top += (h0 && (h1 || h2 || h3)) ? kDualRays : 0;
    *top = ch.y;
    top += (h1 && (h2 || h3)) ? kDualRays : 0;
    *top = ch.z;
    top += (h2 && h3) ? kDualRays : 0;
    if (top > stk_cap) {  // stack full: the rest of this traversal is void, the linear scan decides
      top = stk + stack_cap * kDualRays;
      T.nc = 5;
    }
    T.top = top;
  } else if (T.top == stk) {
    T.node = kTravDone;
  } else {
    T.top -= kDualRays;
    T.node = *T.top;
  }
}

// The FP64 leaf test (yk_render_persistent's, one sphere per leaf: kLeafCapF64), then the pop
__device__ __forceinline__ void dual_leaf(DTrav& T, const KernelArgs& ka, SphereGeo sg, uint32_t id, uint32_t cnt,
                                          v3 o, v3 d, int32_t* stk, uint32_t& n_test, uint32_t& n_dpos) {
  static_assert(kLeafCapF64 == 1, "the FP64 leaf test handles one sphere");
  if (cnt != 0) do {
    ++n_test;
    const v3 oc = {o.x - sg.cx, o.y - sg.cy, o.z - sg.cz};
    const double hb = ykd::dot(oc, d);
    const double c = ykd::len2(oc) - sg.rr;
    const double disc = hb * hb - T.a * c;
    if (disc < 0) continue;
    ++n_dpos;
    const double sq = ykd::sqrt_bound(disc);
    const double r1 = (-hb - sq) * T.ia, r2 = (-hb + sq) * T.ia;
    const double m = (fabs(hb) + sq) * T.ia * 0x1p-34 + 0x1p-1000;
    if (r2 + m < ka.t_min) continue;
    const double lb = fmax(ka.t_min, r1 - m);
    const double ub = (r1 - m >= ka.t_min) ? r1 + m : ((r2 - m >= ka.t_min) ? r2 + m : INFINITY);
    // U* kept as ustar_f = RN(RN(U*) (1 + 2^-18)) only: RN(lb) > ustar_f implies lb > U*, so the
    // float test drops only spheres the double test would drop (all bounds >= 0, monotone
    // rounding), and the minimum of RN(RN(ub) (1 + 2^-18)) is the value at the minimum ub
    const float lbf = (float)lb;
    if (!(lbf <= T.ustar_f)) continue;
    const float ubf = (float)ub * (1.0f + 0x1p-18f);
    if (ubf < T.ustar_f) T.ustar_f = ubf;
    uint32_t c0 = T.c01 & 0xffffu, c1 = T.c01 >> 16, c2 = T.c23 & 0xffffu, c3 = T.c23 >> 16;
    float l0 = T.l0, l1 = T.l1, l2 = T.l2, l3 = T.l3;
    if (T.nc == 4) {
      uint32_t m2 = 0;
      const uint32_t d0 = c0, d1 = c1, d2 = c2, d3 = c3;
      const float e0 = l0, e1 = l1, e2 = l2, e3 = l3;
      if (e0 <= T.ustar_f) { YK_CAND_SET(m2, d0, e0); ++m2; }
      if (e1 <= T.ustar_f) { YK_CAND_SET(m2, d1, e1); ++m2; }
      if (e2 <= T.ustar_f) { YK_CAND_SET(m2, d2, e2); ++m2; }
      if (e3 <= T.ustar_f) { YK_CAND_SET(m2, d3, e3); ++m2; }
      T.nc = m2;
    }
    if (T.nc < 4) {
      c3 = c2, l3 = l2, c2 = c1, l2 = l1, c1 = c0, l1 = l0;
      c0 = id, l0 = lbf;
      ++T.nc;
    } else {
      T.nc = 5;
    }
    T.c01 = c0 | (c1 << 16), T.c23 = c2 | (c3 << 16);
    T.l0 = l0, T.l1 = l1, T.l2 = l2, T.l3 = l3;
  } while (0);
  if (T.top == stk) {
    T.node = kTravDone;
  } else {
    T.top -= kDualRays;
    T.node = *T.top;
  }
}

// The survivors' exact roots after the traversal (or the linear scan), as yk_render_persistent
__device__ __forceinline__ Hit dual_resolve(DTrav& T, const KernelArgs& ka, const SphereGeo* geo, bool alive, v3 o,
                                            v3 d, uint32_t& n_test, uint32_t& n_lin) {
  Hit hit{INFINITY, -1, 0, 0, 0, 0};
  if (!alive) return hit;
  bool linear = T.linear || T.nc > 4;
  if (!linear) {
    const bool a_ok = ykd::div_range(T.a);
    const double ra = (T.nc > 0 && a_ok) ? ykd::rcp_refined(T.a) : 0.0;
    if (T.nc > 0 && T.l0 <= T.ustar_f) exact_candidate(geo, dual_cand(T, 0), o, d, T.a, ra, a_ok, ka.t_min, hit);
    if (T.nc > 1 && T.l1 <= T.ustar_f) exact_candidate(geo, dual_cand(T, 1), o, d, T.a, ra, a_ok, ka.t_min, hit);
    if (T.nc > 2 && T.l2 <= T.ustar_f) exact_candidate(geo, dual_cand(T, 2), o, d, T.a, ra, a_ok, ka.t_min, hit);
    if (T.nc > 3 && T.l3 <= T.ustar_f) exact_candidate(geo, dual_cand(T, 3), o, d, T.a, ra, a_ok, ka.t_min, hit);
  }
  if (linear) {
    hit = scan_linear(ka.geo, ka.nspheres, o, d, ka.t_min);
    n_test += hit.tests;
    ++n_lin;
  }
  return hit;
}

// Refill of one path slot: yk_render_persistent's claim (one wave-uniform reserve for both paths)
template <class Gen>
__device__ __forceinline__ void dual_claim(const KernelArgs& ka, DPath<Gen>& P, uint32_t lane, uint32_t& res_base,
                                           uint32_t& res_left) {
  const bool want = P.live && !P.in_path;
  if (claim_slots(ka, !want, lane, P.slot, res_base, res_left)) P.live = false;
}

// A path's start from its slot (source.cpp:154-165): the pixel and StartRec loads were issued
// by the caller (dual_start_load); yk_render_persistent's start, operation for operation
template <int kMode, class Gen>
__device__ __forceinline__ void dual_start(const KernelArgs& ka, DPath<Gen>& P, bool start, uint32_t qpix, uint4 rq0,
                                           uint4 rq1, uint4 rq2, uint4 rq3) {
  constexpr bool kRandomSeed = (kMode & 2) != 0;
  if (!start) return;
  const uint32_t s = ka.s0 + fdiv(P.slot, ka.nps_m, ka.nps_sh);
  const uint32_t tr = fdiv(qpix, ka.w_m, ka.w_sh);
  const uint32_t x = tile_col_x(ka.col_begin, ka.col_stride, ka.col_band, qpix - tr * ka.Wt);
  const uint32_t y = tile_row_y(ka.row_begin, ka.row_stride, ka.band_log2, tr);
  const uint32_t seed = ykd::sample_seed(kRandomSeed ? 1u : 0u, ka.seed_key, ka.seed0, y, x, ka.W, ka.spp, s);
  StartRec r;
  __builtin_memcpy((char*)&r, &rq0, 16);
  __builtin_memcpy((char*)&r + 16, &rq1, 16);
  __builtin_memcpy((char*)&r + 32, &rq2, 16);
  __builtin_memcpy((char*)&r + 48, &rq3, 16);
  if (r.j != kNoStart) {
    P.g.seed = seed;
    P.g.a0 = r.a0;
    P.g.a1 = r.a1;
    P.g.b = r.b;
    P.g.j = r.j;
    P.o = v3{r.ox, r.oy, r.oz};
    P.d = v3{r.dx, r.dy, r.dz};
  } else {
    const bool lens = ka.cam.lens_radius > 0;
    rng_start_full(P.g, seed);
    const double uc = ykd::canonical<true>(P.g);
    const double vc = ykd::canonical<true>(P.g);
    double px = 0, py = 0;
    if (lens) {
      do {
        px = ykd::uniform(P.g, -1, 1);
        py = ykd::uniform(P.g, -1, 1);
      } while (!(px * px + py * py < 1.0));
    }
    camera_ray(ka.cam, ka.w_d, ka.inv_w, ka.h_d, ka.inv_h, ka.H, x, y, uc, vc, lens, px, py, P.o, P.d);
  }
  P.depth = ka.max_depth;
  P.nstk = 0;
  P.in_path = true;
}

// Shading of one path's segment and its end (yk_render_persistent's (b) and unwind blocks,
// verbatim in operation order): material-uniform canonical block, one normalisation, one second
// Newton square root; the attenuation unwind and the colour store when the path ends.
template <bool kCount, class Gen>
__device__ __forceinline__ void dual_shade_end(const KernelArgs& ka, DPath<Gen>& P, bool alive, const Hit& hit,
                                               const SphereGeo* geo, const SphereMat* mat, uint32_t& n_ncall,
                                               uint32_t& n_nit, uint32_t& n_fb, uint32_t& n_lamb, uint32_t& n_metal,
                                               uint32_t& n_fuzz, uint32_t& n_diel) {
  bool ended = P.in_path && !alive;
  double L_r = 0, L_g = 0, L_b = 0;
  Gen& g = P.g;
  if (alive) {
    const int hid = hit.hid;
    const double T = hit.T;
    SphereGeo sg{0, 0, 0, 0};
    SphereMat m{};
    v3 p{0, 0, 0}, nrm{0, 0, 0};
    bool front = false;
    if (hid >= 0) {
      sg = geo[hid];
      m = mat[hid];
      p = ykd::add(P.o, ykd::mul(P.d, T));
      const v3 outward = ykd::divs_fast_r(ykd::sub(p, v3{sg.cx, sg.cy, sg.cz}), m.radius, m.inv_r);
      front = ykd::dot(P.d, outward) < 0;
      nrm = front ? outward : ykd::neg(outward);
    }
    const bool lamb = hid >= 0 && m.kind == YK_MATERIAL_LAMBERTIAN;
    const bool fuzzy = hid >= 0 && m.kind == YK_MATERIAL_METAL && m.fuzz > 0;
    const bool diel = hid >= 0 && m.kind == YK_MATERIAL_DIELECTRIC;
    const bool spec = diel && ykd::rng_can_speculate(g);
    const Gen saved = g;
    const uint32_t ncan = lamb ? 3u : (fuzzy ? 4u : (spec ? 1u : 0u));
    double c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    if (__ballot(ncan > 0 && !ykd::rng_lazy_ok(g, 2 * ncan)) == 0) {
      if (ncan > 0) c0 = ykd::canonical<true>(g);
      if (ncan > 1) c1 = ykd::canonical<true>(g);
      if (ncan > 2) c2 = ykd::canonical<true>(g);
      if (ncan > 3) c3 = ykd::canonical<true>(g);
    } else {
      if (ncan > 0) c0 = ykd::canonical(g);
      if (ncan > 1) c1 = ykd::canonical(g);
      if (ncan > 2) c2 = ykd::canonical(g);
      if (ncan > 3) c3 = ykd::canonical(g);
    }
    const v3 rv = lamb ? v3{ykd::uniform_of(c0, -1, 1), ykd::uniform_of(c1, -1, 1), ykd::uniform_of(c2, -1, 1)}
                       : v3{ykd::uniform_of(c1, -1, 1), ykd::uniform_of(c2, -1, 1), ykd::uniform_of(c3, -1, 1)};
    const v3 vn = lamb ? rv : P.d;
    const double len = ykd::nsqrt_c(ykd::len2(vn), n_ncall, n_nit);
    const v3 un = ykd::divs_fast(vn, len);
    double ct = 0;
    if (diel) {
      ct = ykd::dot(ykd::neg(un), nrm);
      if (!(ct < 1.0)) ct = 1.0;
    }
    double sq2 = 0;
    if (fuzzy || diel) sq2 = ykd::nsqrt_c(fuzzy ? ykd::len2(rv) : 1.0 - ct * ct, n_ncall, n_nit);
    if (hid < 0) {
      const double t = (un.y + 1.0) / 2;
      L_r = (1.0 - t) * 1.0 + t * 0.5;
      L_g = (1.0 - t) * 1.0 + t * 0.7;
      L_b = (1.0 - t) * 1.0 + t * 1.0;
      ended = true;
    } else {
      bool scattered = true, push = true;
      v3 nd;
      if (m.kind == YK_MATERIAL_LAMBERTIAN) {
        if (kCount) ++n_lamb;
        nd = ykd::add(nrm, un);
        if (ykd::near_zero(nd)) nd = nrm;
      } else if (m.kind == YK_MATERIAL_METAL) {
        if (kCount) ++n_metal;
        nd = ykd::reflect(un, nrm);
        if (fuzzy) {
          if (kCount) ++n_fuzz;
          const double k = ykd::uniform_of(c0, 0.01, 0.99);
          const v3 ru = ykd::divs_fast(rv, sq2);
          nd = ykd::add(nd, ykd::mul(ykd::mul(ru, k), m.fuzz));
        }
        scattered = ykd::dot(nd, nrm) > 0;
      } else {
        if (kCount) ++n_diel;
        push = false;
        const double ratio = front ? (1.0 / m.ior) : m.ior;
        const v3 unit = un;
        const double sn = sq2;
        const bool cannot = ratio * sn > 1.0;
        double u = 0;
        if (cannot) {
          if (spec) g = saved;
        } else {
          u = spec ? ykd::uniform_of(c0, 0, 1) : ykd::uniform(g, 0, 1);
        }
        if (cannot || ykd::reflectance(ct, ratio) > u) {
          nd = ykd::reflect(unit, nrm);
        } else {
          const v3 perp = ykd::mul(ykd::add(unit, ykd::mul(nrm, ct)), ratio);
          const double pl = 1.0 - ykd::len2(perp);
          nd = ykd::add(perp, ykd::mul(nrm, -ykd::nsqrt_c(pl < 0 ? -pl : pl, n_ncall, n_nit)));
        }
      }
      if (!scattered) {
        ended = true;
      } else {
        if (push) {
          if (P.nstk >= kStackRegs) P.id_spill[P.nstk - kStackRegs] = (uint16_t)(P.st3 >> 16);
          P.st3 = (P.st3 << 16) | (P.st2 >> 16);
          P.st2 = (P.st2 << 16) | (P.st1 >> 16);
          P.st1 = (P.st1 << 16) | (P.st0 >> 16);
          P.st0 = (P.st0 << 16) | (uint32_t)hid;
          ++P.nstk;
        }
        P.o = p;
        P.d = nd;
        --P.depth;
      }
    }
  }
  if (ended) {
    while (P.nstk > 0) {
      const uint32_t id = P.st0 & 0xffffu;
      P.st0 = (P.st0 >> 16) | (P.st1 << 16);
      P.st1 = (P.st1 >> 16) | (P.st2 << 16);
      P.st2 = (P.st2 >> 16) | (P.st3 << 16);
      P.st3 = (P.st3 >> 16) | (P.nstk > kStackRegs ? ((uint32_t)P.id_spill[P.nstk - kStackRegs - 1] << 16) : 0u);
      --P.nstk;
      const SphereMat mm = mat[id];
      L_r = mm.ar * L_r;
      L_g = mm.ag * L_g;
      L_b = mm.ab * L_b;
    }
    if (ykd::mt_used_fallback(g)) ++n_fb;
    colour_store(ka.col, P.slot, L_r, L_g, L_b);
    P.in_path = false;
  }
}

// kMode as yk_render_persistent's (bit 0: work counters, bit 1: random-device seeding); mt19937
// only (its StartRecs; xor128 keeps its own instances)
template <bool kSceneInLds, int kMode>
__global__ __launch_bounds__(kDualBlock)
#ifndef YK_DUAL_WAVES
#define YK_DUAL_WAVES 2
#endif
__attribute__((amdgpu_waves_per_eu((kMode & 1) ? 1 : YK_DUAL_WAVES, 8)))
#ifdef YK_DUAL_VGPRS
__attribute__((amdgpu_num_vgpr(YK_DUAL_VGPRS / 2)))  // (gfx950 counts the unified register file: x2)
#endif
void yk_render_dual(KernelArgs ka) {
  constexpr bool kCount = (kMode & 1) != 0;
  using Gen = ykd::MtLane;
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const char* __restrict__ nodes = (const char*)ka.nodes;
  const SphereGeo* __restrict__ leaf_geo = ka.leaf_geo;
  const uint32_t* __restrict__ leaf_ids = ka.leaf_ids;
  const SphereGeo* __restrict__ geo = ka.geo;
  const SphereMat* __restrict__ mat = ka.mat;
  if (kSceneInLds) {
    const uint4* src[5] = {(const uint4*)ka.nodes, (const uint4*)ka.leaf_geo, (const uint4*)ka.leaf_ids,
                           (const uint4*)ka.geo, (const uint4*)ka.mat};
    const uint32_t off[5] = {0u, ka.lds_geo_off, ka.lds_ids_off, ka.lds_tgeo_off, ka.lds_mat_off};
    const uint32_t n16[5] = {(ka.n_nodes * (uint32_t)sizeof(DevNode) + 15u) / 16u, ka.nspheres * 2u,
                             (ka.nspheres + 3u) / 4u, ka.nspheres * 2u, ka.nspheres * 4u};
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      uint4* dst = (uint4*)(smem + off[k]);
      for (uint32_t i = threadIdx.x; i < n16[k]; i += kDualBlock) dst[i] = src[k][i];
    }
    __syncthreads();
    nodes = smem;
    leaf_geo = (const SphereGeo*)(smem + ka.lds_geo_off);
    leaf_ids = (const uint32_t*)(smem + ka.lds_ids_off);
    geo = (const SphereGeo*)(smem + ka.lds_tgeo_off);
    mat = (const SphereMat*)(smem + ka.lds_mat_off);
  }
  // traversal stacks: ray A of this lane at column threadIdx.x, ray B at threadIdx.x + kDualBlock,
  // entries kDualRays words apart
  int32_t* const stkA = (int32_t*)(smem + ka.lds_stack_off) + threadIdx.x;
  int32_t* const stkB = stkA + kDualBlock;
  int32_t* const capA = stkA + ka.stack_cap * kDualRays;
  int32_t* const capB = stkB + ka.stack_cap * kDualRays;
#if YK_RENDER_PRIO
  __builtin_amdgcn_s_setprio(YK_RENDER_PRIO);
#endif
  YK_CLOCK_BEGIN(ka);

  DPath<Gen> A, B;
  rng_init(A.g, ka, 2 * gid);
  rng_init(B.g, ka, 2 * gid + 1);
  A.id_spill = ka.id_scratch + (size_t)(2 * gid) * ka.id_stride;
  B.id_spill = ka.id_scratch + (size_t)(2 * gid + 1) * ka.id_stride;
  A.slot = B.slot = 0;
  A.depth = B.depth = 0;
  A.nstk = B.nstk = 0;
  A.st0 = A.st1 = A.st2 = A.st3 = 0;
  B.st0 = B.st1 = B.st2 = B.st3 = 0;
  A.o = A.d = B.o = B.d = v3{0, 0, 0};
  A.in_path = B.in_path = false;
  A.live = B.live = true;

  uint32_t n_seg = 0, n_test = 0, n_sqrt = 0, n_fb = 0, n_node = 0, n_lin = 0, n_ncall = 0, n_nit = 0;
  uint32_t n_dpos = 0, n_lamb = 0, n_metal = 0, n_fuzz = 0, n_diel = 0;
  uint32_t res_base = 0, res_left = 0;
  const float tmin_lo = __double2float_rd(ka.t_min) * (1.0f - 0x1p-17f);

  for (;;) {
    // ---- refill: both path slots from the wave's reserve; the lane leaves when neither has a
    // path and the launch has no slots left
    dual_claim(ka, A, lane, res_base, res_left);
    dual_claim(ka, B, lane, res_base, res_left);
    if (!A.live && !B.live) break;

    // ---- starts: both paths' pixel and StartRec loads issued together, waited for once
    bool sA = !A.in_path && A.live, sB = !B.in_path && B.live;
    uint32_t qA = 0, qB = 0;
    uint4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0, b0 = a0, b1 = a0, b2 = a0, b3 = a0;
    if (sA) {
      const uint32_t sl = fdiv(A.slot, ka.nps_m, ka.nps_sh);
      qA = ka.order[A.slot - sl * ka.npix_slots];
      const uint4* rp = (const uint4*)ka.start + 4u * A.slot;
      a0 = rp[0], a1 = rp[1], a2 = rp[2], a3 = rp[3];
    }
    if (sB) {
      const uint32_t sl = fdiv(B.slot, ka.nps_m, ka.nps_sh);
      qB = ka.order[B.slot - sl * ka.npix_slots];
      const uint4* rp = (const uint4*)ka.start + 4u * B.slot;
      b0 = rp[0], b1 = rp[1], b2 = rp[2], b3 = rp[3];
    }
    asm volatile("" ::"v"(a0.x), "v"(a0.y), "v"(a0.z), "v"(a0.w), "v"(a1.x), "v"(a1.y), "v"(a1.z), "v"(a1.w),
                 "v"(a2.x), "v"(a2.y), "v"(a2.z), "v"(a2.w), "v"(a3.x), "v"(a3.y), "v"(a3.z), "v"(a3.w), "v"(qA));
    asm volatile("" ::"v"(b0.x), "v"(b0.y), "v"(b0.z), "v"(b0.w), "v"(b1.x), "v"(b1.y), "v"(b1.z), "v"(b1.w),
                 "v"(b2.x), "v"(b2.y), "v"(b2.z), "v"(b2.w), "v"(b3.x), "v"(b3.y), "v"(b3.z), "v"(b3.w), "v"(qB));
    sA = sA && qA != kNoPixel;  // an empty slot of an edge block: another claim next trip
    sB = sB && qB != kNoPixel;
    dual_start<kMode>(ka, A, sA, qA, a0, a1, a2, a3);
    dual_start<kMode>(ka, B, sB, qB, b0, b1, b2, b3);
    if (kCount && (ka.flags & kFlagTrace)) {
      if (A.in_path) trace_ray(ka, A.slot, ka.max_depth - A.depth, A.o, A.d);
      if (B.in_path) trace_ray(ka, B.slot, ka.max_depth - B.depth, B.o, B.d);
    }

    // ---- closest hits of both rays: one traversal loop, one node of each per trip
    const bool aliveA = A.in_path && A.depth != 0, aliveB = B.in_path && B.depth != 0;
    n_seg += (aliveA ? 1u : 0u) + (aliveB ? 1u : 0u);
    DTrav TA, TB;
    dual_trav_setup(TA, ka, nodes, aliveA, A.o, A.d, stkA);
    dual_trav_setup(TB, ka, nodes, aliveB, B.o, B.d, stkB);
    for (;;) {
      if (TA.node == kTravDone && TB.node == kTravDone) break;
      const bool vA = TA.node >= 0, vB = TB.node >= 0;
      // issue both rays' reads: an inner node's planes and child codes, or a leaf's sphere
      f4 pA0, pA1, pA2, pA3, pA4, pA5, pB0, pB1, pB2, pB3, pB4, pB5;
      int4 chA, chB;
      uint32_t idA = 0, idB = 0;
      if (vA) {
        const int32_t nd = TA.node;
        pA0 = *(const f4*)(TA.px + nd), pA1 = *(const f4*)(TA.px + nd + 16);
        pA2 = *(const f4*)(TA.py + nd), pA3 = *(const f4*)(TA.py + nd + 16);
        pA4 = *(const f4*)(TA.pz + nd), pA5 = *(const f4*)(TA.pz + nd + 16);
        chA = *(const int4*)(nodes + nd + 144);
      } else if (TA.node != kTravDone) {
        const uint32_t first = (~(uint32_t)TA.node) >> 4;
        pA0 = *(const f4*)&leaf_geo[first];
        pA1 = *((const f4*)&leaf_geo[first] + 1);
        idA = leaf_ids[first];
      }
      if (vB) {
        const int32_t nd = TB.node;
        pB0 = *(const f4*)(TB.px + nd), pB1 = *(const f4*)(TB.px + nd + 16);
        pB2 = *(const f4*)(TB.py + nd), pB3 = *(const f4*)(TB.py + nd + 16);
        pB4 = *(const f4*)(TB.pz + nd), pB5 = *(const f4*)(TB.pz + nd + 16);
        chB = *(const int4*)(nodes + nd + 144);
      } else if (TB.node != kTravDone) {
        const uint32_t first = (~(uint32_t)TB.node) >> 4;
        pB0 = *(const f4*)&leaf_geo[first];
        pB1 = *((const f4*)&leaf_geo[first] + 1);
        idB = leaf_ids[first];
      }
      if (kCount) n_node += (vA ? 1u : 0u) + (vB ? 1u : 0u);
      // then A's visit or leaf while B's reads are in flight, then B's
      if (vA) {
        dual_advance(TA, dual_slots(TA, tmin_lo, pA0, pA1, pA2, pA3, pA4, pA5), chA, stkA, capA, ka.stack_cap);
      } else if (TA.node != kTravDone) {
        SphereGeo sg;
        __builtin_memcpy((char*)&sg, &pA0, 16);
        __builtin_memcpy((char*)&sg + 16, &pA1, 16);
        dual_leaf(TA, ka, sg, idA, (~(uint32_t)TA.node) & 15u, A.o, A.d, stkA, n_test, n_dpos);
      }
      if (vB) {
        dual_advance(TB, dual_slots(TB, tmin_lo, pB0, pB1, pB2, pB3, pB4, pB5), chB, stkB, capB, ka.stack_cap);
      } else if (TB.node != kTravDone) {
        SphereGeo sg;
        __builtin_memcpy((char*)&sg, &pB0, 16);
        __builtin_memcpy((char*)&sg + 16, &pB1, 16);
        dual_leaf(TB, ka, sg, idB, (~(uint32_t)TB.node) & 15u, B.o, B.d, stkB, n_test, n_dpos);
      }
    }
    Hit hA = dual_resolve(TA, ka, geo, aliveA, A.o, A.d, n_test, n_lin);
    Hit hB = dual_resolve(TB, ka, geo, aliveB, B.o, B.d, n_test, n_lin);
    n_sqrt += hA.sqrts + hB.sqrts;
    n_ncall += hA.ncalls + hB.ncalls;
    n_nit += hA.nits + hB.nits;

    // ---- shading and path ends, A then B
    dual_shade_end<kCount>(ka, A, aliveA, hA, geo, mat, n_ncall, n_nit, n_fb, n_lamb, n_metal, n_fuzz, n_diel);
    dual_shade_end<kCount>(ka, B, aliveB, hB, geo, mat, n_ncall, n_nit, n_fb, n_lamb, n_metal, n_fuzz, n_diel);
  }

  YK_CLOCK_END(ka);
  if (kCount) {
    atomicAdd(&ka.counters[0], (unsigned long long)n_seg);
    atomicAdd(&ka.counters[1], (unsigned long long)n_test);
    atomicAdd(&ka.counters[2], (unsigned long long)n_sqrt);
    atomicAdd(&ka.counters[4], (unsigned long long)n_node);
    atomicAdd(&ka.counters[5], (unsigned long long)n_lin);
    atomicAdd(&ka.counters[6], (unsigned long long)n_ncall);
    atomicAdd(&ka.counters[7], (unsigned long long)n_nit);
    atomicAdd(&ka.counters[24], (unsigned long long)n_dpos);
    atomicAdd(&ka.counters[25], (unsigned long long)n_lamb);
    atomicAdd(&ka.counters[26], (unsigned long long)n_metal);
    atomicAdd(&ka.counters[27], (unsigned long long)n_fuzz);
    atomicAdd(&ka.counters[28], (unsigned long long)n_diel);
  }
  if (n_fb) atomicAdd(&ka.counters[3], (unsigned long long)n_fb);
}

// The dual instance for (scene in LDS, kMode & 3)
RenderKernel dual_kernel(bool lds, int mode) {
  static const RenderKernel k[8] = {yk_render_dual<false, 0>, yk_render_dual<false, 1>, yk_render_dual<false, 2>,
                                    yk_render_dual<false, 3>, yk_render_dual<true, 0>,  yk_render_dual<true, 1>,
                                    yk_render_dual<true, 2>,  yk_render_dual<true, 3>};
  return k[(lds ? 4 : 0) + (mode & 3)];
}
