// ykgpu_render.hip — the per-pixel sampling loop of UECRayTracing on gfx950 (MI355X), and the
// C-ABI (include/ykgpu.h) around it.
//
// Replaces /root/reference/source.cpp:122-172 (for_each over (row,col) → transform_reduce over
// samples → to_color3b) and the recursion of yk/raytracer.hpp:19-37.
//
// Execution model:
//   * a render call is a sequence of LAUNCHES of K samples per pixel (a synced call: 4, 8, 16,
//     then at most kLaunchSpp = 32 for the frame: 1920x1080x512 is 4, 8, 16, 14 x 32, 18, 18; a
//     call enqueued while the previous one still runs: kLaunchSppOv = 64, 8 x 64).  Per launch: yk_mt_warmup (second
//     stream: every sample's mt19937 seeding walk and its start draws — jitter and lens — and
//     camera ray, as a StartRec), yk_render_persistent (the paths, on one of two top-priority
//     streams), yk_reduce_samples (the reference's strictly sequential per-pixel sum and
//     to_color3b, third stream).  Back-to-back calls overlap (launches numbered across calls).
//   * yk_render_persistent is one persistent grid of 768-thread workgroups, one per CU (12 waves,
//     3 per SIMD at 112 VGPRs, beside three 48-VGPR warm-up waves), with
//     the scene (BVH, geometry and material tables) in LDS, over SAMPLE SLOTS: a lane runs one path at a
//     time, one SEGMENT (closest hit + scatter) per trip round the loop, writes the sample's
//     colour when the path ends and takes the next slot from a wave-level reserve (one atomic
//     per 512 slots) — active-lane refill, so no lane idles while the launch has slots.
//   * the colour of a path is attenuation_1 * (attenuation_2 * (... * L)): double
//     multiplication does not associate, so the lane keeps the ids of the scattering spheres
//     on a small stack (8 in registers, the rest in a per-lane global spill) and multiplies
//     back to front at the end (raytracer.hpp:31).
//   * closest hit: a 4-wide BVH in LDS culls conservatively in float, the candidates' roots
//     are evaluated with the reference's exact arithmetic, ties to the later tuple index
//      — the result equals the reference's ordered scan bit for bit.
//   * every operation several lane kinds need runs once per trip for all of them (shared
//     canonical block, normalisation and second square root in shading): a wave pays for each
//     branch any of its lanes takes ("Uniform work per trip").
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <random>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/ykgpu.h"
#include "yk_bvh.hpp"
#include "yk_device.hpp"
#include "yk_device_f32.hpp"
#include "yk_stamps.hpp"

using ykd::v3;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

#define YK_HIP(call)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fail(e_ == hipErrorOutOfMemory ? YK_ERR_NOMEM : YK_ERR_DEVICE,               \
                  std::string(#call) + ": " + hipGetErrorString(e_));                     \
  } while (0)

// Geometry of one sphere, as the closest-hit scan reads it (32 B: one scalar x8 load).
// rr = radius*radius computed on the host with the same IEEE multiply as sphere.hpp:33.
struct alignas(32) SphereGeo {
  double cx, cy, cz, rr;
};
// Shading data, read once per segment by the lane that hit the sphere.
struct alignas(16) SphereMat {
  double ar, ag, ab, fuzz;
  double radius, ior;
  uint32_t kind;
  float inv_rf;  // ykf::rcp_refined((float)radius) (FP32 kernel), computed on the device by yk_mat_prep
  double inv_r;  // ykd::rcp_refined(radius), computed on the device by yk_mat_prep
};
static_assert(sizeof(SphereMat) == 64, "SphereMat layout");

// One 768-thread workgroup per CU (12 waves, 3 per SIMD): the scene is copied into LDS once per
// CU instead of once per 256-thread block, which leaves room for the shading tables (sphere
// geometry and materials in tuple order) beside the BVH and the traversal stacks.  The fourth
// wave slot of each SIMD (128 of its 512 VGPRs) is left to the yk_mt_warmup waves, which run the
// next launch's seed walks in the render's idle issue cycles.  (1024 threads, 4 render waves per
// SIMD: the node loop is bound by LDS latency, so the render alone runs 4% faster — 184 vs 192 ms
// per 512-spp frame without the walks — but the walks can no longer overlap: 218 vs 215 ms.)
#ifndef YK_BLOCK
#define YK_BLOCK 768
#endif
#ifndef YK_WAVES_PER_EU
#define YK_WAVES_PER_EU 0
#endif
constexpr int kBlock = YK_BLOCK;
// The xor128 instances draw no seed walks, so nothing needs the fourth wave slot of a SIMD: they
// run 1024-thread workgroups (4 render waves per SIMD; the node loop is bound by LDS latency, so
// the fourth wave pays)
#ifndef YK_BLOCK_X128
#define YK_BLOCK_X128 1024
#endif
constexpr int kBlockX128 = YK_BLOCK_X128;
template <int kMode>
constexpr int mode_block() {
  return (kMode & 4) ? kBlockX128 : kBlock;
}
constexpr int block_of(bool x128) { return x128 ? kBlockX128 : kBlock; }
#ifndef YK_RENDER_PRIO
#define YK_RENDER_PRIO 1
#endif
// the visit's slab constants as one op_sel-read register pair per axis and bound (yk_slab.hpp):
// round 4: FP64 123 -> 115 VGPRs and no faster (512 spp 173.9 -> 174.2 ms), FP32 125 -> 111 VGPRs
// and faster (195.3 -> 190.1 ms, profiles/r04_ab/f32/).  Round 6, on the branch-free visit: FP64
// 128 -> 114 VGPRs, bench -0.7% (the SIMD's spare registers take a third warm-up wave,
// profiles/r06_ab/vgpr/), so both kernels now read slab pairs.
// YK_SLAB_PAIRS sets both (A/B).  (Round 4's two-paths-per-lane kernel, which lost its A/B, is
// kept as a patch beside its evidence: profiles/r04_ab/dual/yk_dual.patch.)
#ifdef YK_SLAB_PAIRS
#define YK_SLAB_PAIRS_F64 YK_SLAB_PAIRS
#define YK_SLAB_PAIRS_F32 YK_SLAB_PAIRS
#endif
#ifndef YK_SLAB_PAIRS_F64
#define YK_SLAB_PAIRS_F64 1
#endif
#ifndef YK_SLAB_PAIRS_F32
#define YK_SLAB_PAIRS_F32 1
#endif
// (Tried and removed in round 4, DESIGN.md §4.1: the FP32 slow-axis bound folded into the slow
// axis' far-plane FMA, +2.3%; the slow-axis read skipped in waves without a slow-axis ray, +3.8%.)
using DevNode = ykbvh::WideNode;  // 4-wide BVH nodes (yk_bvh.hpp)
constexpr int kCounters = 32;  // [16..18]: timeline, [19..22]: diag (stamp builds), [24..31]: work
// Spheres per BVH leaf the kernels' leaf code handles: the FP64 leaf test is loop-free for one
// sphere, the FP32 leaf loop is unrolled for two.  ykgpu_set_scene builds the trees with these
// as ykbvh::Options::max_leaf and upload_tree rejects a tree with a larger leaf (its extra spheres
// would be skipped silently).
constexpr uint32_t kLeafCapF64 = 1, kLeafCapF32 = 2;
constexpr uint32_t kStackRegs = 8;  // attenuation ids kept in registers (4 x 2 x u16)
// FP64 node visit without a branch (round 6): the stack's bottom entry holds the empty leaf (a
// sentinel), so "no slot entered" pops unconditionally and every lane of the visit runs the same
// instructions; a lane's run of interior nodes is a loop of its own (while-while), the entry below
// the top read with the planes.  2: the loop variable is the address of that entry (constant DS
// offsets for it and the pushes).  0: the round-5 visit with its push / pop branches (A/B).
// 512 spp, same box (profiles/r06_ab/nodebf/): 0 -> 1: bench 163.0 -> 159.5 ms; 2 = 1.
#ifndef YK_NODE_BF
#define YK_NODE_BF 2
#endif
// the FP64 stack sized to the tree's proven depth (3 x wide depth + 1 entries) where LDS allows,
// its overflow check then skipped (a scalar branch on KernelArgs::stack_check): bench 159.0 ->
// 156.2 ms on top of YK_NODE_BF (0: always checked, A/B)
// the FP64 candidate list's ids as 16-bit halves of two registers (written for the YK_CAND_HD /
// YK_NEAR_CLAMP kernel): the shift-in is one alignbit and one lshl_or instead of four moves, two
// VGPRs freed; bench -0.3...-0.6%, synced -0.4...-0.8%, image hash unchanged (r06_ab/shade/r06ax_*)
#ifndef YK_CAND_PACK
#define YK_CAND_PACK 1
#endif
// ... and its v_rsq_f64, which math::sqrt's start repeats (A/B; 2 VGPRs more)
#ifndef YK_CAND_RSQ
#define YK_CAND_RSQ 0
#endif
// the candidates' refined 1/a from the bounds' 1/a (one Newton step instead of rcp + two; A/B)
#ifndef YK_RA_FROM_IA
#define YK_RA_FROM_IA 0
#endif
// the newest candidate's hb and disc kept from its leaf test, so its exact root skips the second
// discriminant (17 FP64 operations): bench -0.4...-0.6%, synced -0.6%, the headline image's hash
// unchanged, no spill at 112 VGPRs (profiles/r06_ab/shade/r06ar_*)
#ifndef YK_CAND_HD
#define YK_CAND_HD 1
#endif
// the FP64 visit's loop in two copies, with and without the stack check (A/B)
#ifndef YK_VISIT_UNSWITCH
#define YK_VISIT_UNSWITCH 0
#endif
// the FP64 visit's distances from tmin_lo, scaled by kClampScale, the near FMAs clamping to [0, 1]
// in place of the max with tmin_lo: 4 VALU fewer per visit, bench 150.0 -> 147.0 ms, node visits
// unchanged, bit-exact (profiles/r06_ab/shade/r06ai_*)
#ifndef YK_NEAR_CLAMP
#define YK_NEAR_CLAMP 1
#endif
constexpr float kClampScale = 0x1p-24f;
// the FP64 visit's slab min / max two slots per asm block (yk_slab.hpp slab_cull2): one hazard
// pad per visit instead of eight, bench -0.2% (four of four same-box pairs, image hashes equal,
// profiles/r06_ab/shade/r06ag_*)
#ifndef YK_CULL_BLOCK
#define YK_CULL_BLOCK 1
#endif
#ifndef YK_STACK_EXACT
#define YK_STACK_EXACT 1
#endif

// the FP64 dielectric's 1/ior and Schlick r0 (both sides) precomputed on the host: two FP64
// divisions fewer per trip with a glass hit (bench -0.6%, profiles/r06_ab/shade/; 0: A/B)
#ifndef YK_DIEL_PRE
#define YK_DIEL_PRE 1
#endif
// the FP64 unwind without the spill check when no ending lane of the wave spilled, two ids per
// round (bench 156.6 -> 156.0 ms, profiles/r06_ab/unwind/; 0: the round-5 unwind, A/B)
#ifndef YK_UNWIND_FAST
#define YK_UNWIND_FAST 1
#endif
// slot claims: the tail size from a kernel argument and the leader's counter by v_readlane (the
// claim's bookkeeping becomes scalar: 2 VGPRs fewer; 0: A/B)
#ifndef YK_CLAIM_ARGS
#define YK_CLAIM_ARGS 1
#endif
// VGPRs of the production FP64 render instances: 3 render waves x 112 of a SIMD's 512 leave 176, three
// 48-VGPR warm-up waves and a reduce wave (bench -0.4% against the natural 114 -> 120; 104 spills
// and starves the render: +3.4%, profiles/r06_ab/vgpr/); the counting instances keep theirs
#ifndef YK_RENDER_VGPRS
#define YK_RENDER_VGPRS 112
#endif
#ifndef YK_CLAIM
#define YK_CLAIM 512
#endif
constexpr uint32_t kClaim = YK_CLAIM;  // sample slots a wave claims per atomic
// ... and near the end of a launch's slots: when fewer than kClaimTailFactor x kClaim slots per
// wave of the grid remain (as the wave last saw the counter), a wave claims kClaimTail slots at a
// time.  A wave's reserve holds up to kClaim slots (8 samples per lane) when the counter runs
// out, so with full claims to the end some waves still have ~8 samples per lane of work while
// others have none, and every launch drains for that long (0: full claims to the end).
#ifndef YK_CLAIM_TAIL
#define YK_CLAIM_TAIL 64
#endif
#ifndef YK_CLAIM_TAIL_FACTOR
#define YK_CLAIM_TAIL_FACTOR 2
#endif
constexpr uint32_t kClaimTail = YK_CLAIM_TAIL, kClaimTailFactor = YK_CLAIM_TAIL_FACTOR;
static_assert(kClaimTail == 0 || (kClaimTail >= 64 && kClaimTail <= YK_CLAIM), "a tail claim serves a whole wave");
#ifndef YK_WG_HOLD
#define YK_WG_HOLD 0
#endif
// the FP64 lens warm-up's retries drawn after its walks (yk_mt_warmup_defer) for launches of at
// most YK_DEFER_SLOTS slots per warm-up wave (0: the rejection loop in line everywhere)
#ifndef YK_LENS_DEFER
#define YK_LENS_DEFER 1
#endif
#ifndef YK_DEFER_SLOTS
#define YK_DEFER_SLOTS 4096
#endif
constexpr bool kLensDefer = YK_LENS_DEFER != 0;
constexpr uint64_t kDeferSlots = YK_DEFER_SLOTS;
constexpr uint32_t kFlagLinearScan = YK_FLAG_LINEAR_SCAN;
constexpr uint32_t kFlagOneLane = YK_FLAG_ONE_LANE;
constexpr uint32_t kFlagTrace = YK_FLAG_TRACE_RAYS;

// the camera rounded to float once on the host (camera<float>'s members, camera.hpp:10-27), and
// W, H as floats: the FP32 kernel's start converts nothing
struct CamF {
  float origin[3], llc[3], horizontal[3], vertical[3], lens_u[3], lens_v[3];
  float lens_radius, w, h, pad[3];
};
struct KernelArgs {
  yk_camera cam;
  CamF camf;
  uint32_t W, H, spp, max_depth;
  uint32_t seed0, row_begin, row_count, row_stride, band_log2;
  // stack_check: 0 when the FP64 traversal stack holds 3 x (wide depth) + 1 entries, so the
  // branch-free visit cannot overflow it and skips the check (upload_tree)
  uint32_t nspheres, stack_check, flags, id_stride;
  // A launch renders samples [s0, s0 + nsl / npix_slots) of every pixel: sample slot
  // i = s_local * npix_slots + p is sample s0 + s_local of tile pixel order[p].
  uint32_t s0, nsl, npix_slots, seed_mode;  // seed_mode: YK_SEED_*
  uint32_t nps_m, nps_sh, w_m, w_sh;  // fdiv magic numbers of npix_slots and the tile width Wt
  uint64_t seed_key;
  const uint32_t* __restrict__ order;  // p → tile pixel (kNoPixel: empty slot of an edge block)
  uint64_t pad_a;                      // (keeps the argument layout the kernels were tuned with)
  const void* __restrict__ start;      // StartRec per sample slot (mt19937 kernels)
  double t_min;
  double inv_w, inv_h;  // RN(1/W), RN(1/H) for the camera's exact divisions (div_markstein)
  double w_d, h_d;      // W, H as doubles (kernel arguments: no loop-hoisted conversion to hold)
  double origin_bound;  // |o|_inf beyond which the BVH's float culling is not proven sound
  int32_t bvh_root;
  uint32_t n_nodes;
  uint32_t lds_geo_off, lds_ids_off, lds_stack_off, stack_cap;  // stack_cap: entries a lane may hold
  uint32_t lds_tgeo_off, lds_mat_off;  // FP64 kernel: tuple-order geometry / materials in LDS
  const DevNode* __restrict__ nodes;  // child links are byte offsets from nodes
  const SphereGeo* __restrict__ leaf_geo;  // spheres in BVH leaf order
  const uint32_t* __restrict__ leaf_ids;   // leaf slot → tuple index
  const SphereGeo* __restrict__ geo;
  const SphereMat* __restrict__ mat;
  const float4* __restrict__ geo_f;  // FP32 path: (cx, cy, cz, r*r) rounded to float, tuple order
  double* col;                       // sample colours: a record per slot (colour_store)
  uint32_t* pixel_counter;           // sample-slot counter
  uint32_t* mt_scratch;
  uint16_t* id_scratch;
  unsigned long long* counters;  // [segments, sphere_tests, sqrt_calls, mt_fallbacks, nodes]
  double* trace;                 // YK_FLAG_TRACE_RAYS: rays [(q*spp + s)*trace_cap + k][6]
  uint32_t* trace_counts;        //   ray_color calls per sample [q*spp + s]
  uint32_t trace_cap;
  uint32_t claim_tail;  // slots left below which a wave claims kClaimTail: grid x waves x kClaim x factor
  unsigned long long* clk;  // this launch's shader-clock probe (YK_CLOCK_*): 4 words
  // the tile's columns (include/ykgpu.h yk_render_params; the whole width: Wt = W, 0, 1, 0)
  uint32_t Wt, col_begin, col_stride, col_band;
#ifdef YK_DRAIN_DIAG
  uint32_t diag_c, diag_pad;  // the launch's index in its call
#endif
};

// Shader-clock probe of a launch: thread 0 of block 0 stores s_memtime (the shader clock) and
// s_memrealtime (100 MHz) when it starts and when it leaves the loop (vector stores, nothing held
// in registers across the loop) — the clock the launch ran at (ykgpu_get_stats sclk_mhz; the
// per-launch timeline).
#define YK_CLOCK_STAMP(ka, k)                                                              \
  do {                                                                                     \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                                             \
      (ka).clk[(k)] = __builtin_amdgcn_s_memtime();                                        \
      (ka).clk[(k) + 1] = __builtin_amdgcn_s_memrealtime();                                \
    }                                                                                      \
  } while (0)
#define YK_CLOCK_BEGIN(ka) YK_CLOCK_STAMP(ka, 0)
#define YK_CLOCK_END(ka) YK_CLOCK_STAMP(ka, 2)

// Diagnostic builds (YK_DRAIN_DIAG, tools/drain_probe.py): every FP64 render wave records when it
// starts and when it leaves the loop (s_memrealtime, 100 MHz) and where it ran (HW_ID, XCC_ID), per
// launch of the call: the per-launch drain — waves idle in a workgroup that still holds its CU,
// CUs between one launch's workgroup and the next — measured, not modelled
#ifdef YK_DRAIN_DIAG
constexpr uint32_t kDiagLaunches = 64, kDiagBlocks = 512, kDiagWaves = 16;
// per wave: {start, end, HW_ID | XCC_ID << 32}
__device__ unsigned long long yk_wave_times[kDiagLaunches * kDiagBlocks * kDiagWaves * 3];
#define YK_WAVE_STAMP(ka, k)                                                                          \
  do {                                                                                                \
    const uint32_t w_ = threadIdx.x >> 6;                                                             \
    if ((threadIdx.x & 63u) == 0 && (ka).diag_c < kDiagLaunches && blockIdx.x < kDiagBlocks) {        \
      unsigned long long* r_ =                                                                        \
          yk_wave_times + (((size_t)(ka).diag_c * kDiagBlocks + blockIdx.x) * kDiagWaves + w_) * 3;     \
      r_[(k)] = __builtin_amdgcn_s_memrealtime();                                                     \
      if ((k) == 0)                                                                                   \
        r_[2] = (unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 4) |                       \
                ((unsigned long long)__builtin_amdgcn_s_getreg((3 << 11) | 20) << 32);                \
    }                                                                                                 \
  } while (0)
#else
#define YK_WAVE_STAMP(ka, k) ((void)0)
#endif

// -l 3 (raytracer.hpp:21-25): ray k of the path of the lane's sample slot (counting instance)
template <class V>
__device__ __forceinline__ void trace_ray(const KernelArgs& ka, uint32_t slot, uint32_t k, V o, V d) {
  const uint32_t sl = slot / ka.npix_slots, q = ka.order[slot - sl * ka.npix_slots];
  const size_t idx = (size_t)q * ka.spp + ka.s0 + sl;
  if (k < ka.trace_cap) {
    double* r = ka.trace + (idx * ka.trace_cap + k) * 6;
    r[0] = o.x, r[1] = o.y, r[2] = o.z, r[3] = d.x, r[4] = d.y, r[5] = d.z;
  }
  ka.trace_counts[idx] = k + 1;
}

// floor(n / d) for n < 2^31 with the host's magic numbers (fastdiv): ((uint64) n * m) >> sh, where
// l = ceil(log2 d), sh = 31 + l, m = ceil(2^sh / d) < 2^32 — exact for every 31-bit n (the
// round-up error n * (m d - 2^sh) / (d 2^sh) < 2^31 d / (d 2^sh) * d / 2^l <= 1/d).  A runtime
// divisor otherwise costs the ~20-instruction float-reciprocal sequence per division.
__device__ __forceinline__ uint32_t fdiv(uint32_t n, uint32_t m, uint32_t sh) {
  return (uint32_t)(((uint64_t)n * m) >> sh);
}

// Image row of tile row t (include/ykgpu.h yk_render_params: bands of 2^band_log2 rows, every
// row_stride-th band; band_log2 = 0 is the plain strided row set)
__device__ __forceinline__ uint32_t tile_row_y(uint32_t row_begin, uint32_t row_stride, uint32_t band_log2,
                                               uint32_t t) {
  return row_begin + (((t >> band_log2) * row_stride) << band_log2) + (t & ((1u << band_log2) - 1u));
}
// ... and image column of tile column j (bands of 2^col_band columns, every col_stride-th band)
__device__ __forceinline__ uint32_t tile_col_x(uint32_t col_begin, uint32_t col_stride, uint32_t col_band,
                                               uint32_t j) {
  return col_begin + (((j >> col_band) * col_stride) << col_band) + (j & ((1u << col_band) - 1u));
}

struct Hit {
  double T;
  int hid;
  uint32_t tests, sqrts;
  uint32_t ncalls, nits;  // math::sqrt calls / loop iterations
};

// The reference's closest-hit scan verbatim (hittable_list.hpp:32-58 over sphere.hpp:25-48):
// tuple order, t_max shrinking to the last accepted root.  Used for rays the BVH cannot serve
// (degenerate direction, origin beyond the proven float range, candidate-list overflow) and,
// with kFlagLinearScan, as the A/B reference of the BVH path.
__device__ __noinline__ Hit scan_linear(const SphereGeo* __restrict__ geo, uint32_t n, v3 o, v3 d,
                                        double tmin) {
  const double a = ykd::len2(d);
  Hit h{INFINITY, -1, 0, 0, 0, 0};
  for (uint32_t i = 0; i < n; ++i) {
    const SphereGeo sg = geo[i];
    ++h.tests;
    const v3 oc = {o.x - sg.cx, o.y - sg.cy, o.z - sg.cz};
    const double hb = ykd::dot(oc, d);
    const double c = ykd::len2(oc) - sg.rr;
    const double disc = hb * hb - a * c;
    if (disc < 0) continue;
    ++h.sqrts;
    const double sq = ykd::nsqrt_c(disc, h.ncalls, h.nits);
    double root = (-hb - sq) / a;
    if (root < tmin || h.T < root) {
      root = (-hb + sq) / a;
      if (root < tmin || h.T < root) continue;
    }
    h.T = root;
    h.hid = (int)i;
  }
  return h;
}

typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f4 __attribute__((ext_vector_type(4)));

#include "yk_slab.hpp"

__device__ __forceinline__ float safe_rcp(float x) {
  return fabsf(x) > 1e-30f ? 1.0f / x : copysignf(1e30f, x);
}

// Candidate list entry insertion with static register indexing (no scratch).
#define YK_CAND_SET(K, ID, LB) \
  do {                         \
    if ((K) == 0) { c0 = ID; l0 = LB; }       \
    else if ((K) == 1) { c1 = ID; l1 = LB; }  \
    else if ((K) == 2) { c2 = ID; l2 = LB; }  \
    else { c3 = ID; l3 = LB; }                \
  } while (0)

// Exact value of sphere i's root under the reference's acceptance rule, ignoring t_max
// (sphere.hpp:35-39): root1 if root1 >= t_min, else root2 if root2 >= t_min, else none.
// n / a for a root (sphere.hpp:36-38), a's refined reciprocal shared by all candidates; a wave
// with any lane out of range takes the full division (divs_fast's rule)
__device__ __forceinline__ double root_div(double n, double a, double ra, bool a_ok) {
  double q = ykd::div_by(n, a, ra);
  if (__builtin_expect(__ballot(!(a_ok && ykd::num_range(n))) != 0, 0)) q = n / a;
  return q;
}
__device__ __forceinline__ void exact_root(uint32_t i, double hb, double disc, double a, double ra, bool a_ok,
                                           double tmin, Hit& best, const double* rsq = nullptr);
__device__ __forceinline__ void exact_candidate(const SphereGeo* __restrict__ geo, uint32_t i,
                                                v3 o, v3 d, double a, double ra, bool a_ok,
                                                double tmin, Hit& best) {
  const SphereGeo sg = geo[i];
  const v3 oc = {o.x - sg.cx, o.y - sg.cy, o.z - sg.cz};
  const double hb = ykd::dot(oc, d);
  const double c = ykd::len2(oc) - sg.rr;
  const double disc = hb * hb - a * c;
  exact_root(i, hb, disc, a, ra, a_ok, tmin, best);
}
// the root of a candidate whose hb and disc (the reference's, bit for bit) are already known
__device__ __forceinline__ void exact_root(uint32_t i, double hb, double disc, double a, double ra, bool a_ok,
                                           double tmin, Hit& best, const double* rsq) {
  if (disc < 0) return;  // never taken: the candidate passed the same test
  ++best.sqrts;
  // (rsq: v_rsq_f64 of this disc from the leaf test, the instruction math::sqrt's start would repeat)
  const double sq = rsq ? ykd::nsqrt_c_r(disc, *rsq, best.ncalls, best.nits) : ykd::nsqrt_c(disc, best.ncalls, best.nits);
  double r = root_div(-hb - sq, a, ra, a_ok);
  if (r < tmin) {
    r = root_div(-hb + sq, a, ra, a_ok);
    if (r < tmin) return;
  }
  // closest wins; an exact tie goes to the later tuple index (hittable_list.hpp:36-43)
  if (r < best.T || (r == best.T && (int)i > best.hid)) {
    best.T = r;
    best.hid = (int)i;
  }
}

__device__ __forceinline__ v3 ld3(const double* p) { return {p[0], p[1], p[2]}; }

// Processing order: slot p of a call renders tile pixel order[p] (ykgpu_context::order, built on
// the host for the image geometry): 8x8 pixel blocks, so the lanes a wave refills together take
// neighbouring pixels in both directions.  Every pixel's samples are independent of the order.
constexpr uint32_t kNoPixel = 0xffffffffu;

// camera::get_ray (camera.hpp:29-32) for pixel (x, y) from the start's draws: the jitter
// canonicals uc, vc (source.cpp:162-163, (x + U01) / W correctly rounded by Markstein's form with
// the host's RN(1/W), yk_device.hpp) and the thin-lens point (px, py) when the camera has a lens.
// The warm-up and the render kernel's own start (xor128, or a record the warm-up could not
// complete) both call it, so a record's ray is the ray the render would have computed.
__device__ __forceinline__ void camera_ray(const yk_camera& cam, double w_d, double inv_w, double h_d,
                                           double inv_h, uint32_t H, uint32_t x, uint32_t y, double uc,
                                           double vc, bool lens, double px, double py, v3& o, v3& d) {
  const double u = ykd::div_markstein((double)x + ykd::uniform_of(uc, 0, 1), w_d, inv_w);
  const double v = ykd::div_markstein((double)(H - y - 1) + ykd::uniform_of(vc, 0, 1), h_d, inv_h);
  const v3 cam_o = ld3(cam.origin), cam_llc = ld3(cam.lower_left_corner);
  const v3 cam_h = ld3(cam.horizontal), cam_v = ld3(cam.vertical);
  d = ykd::sub(ykd::add(ykd::add(cam_llc, ykd::mul(cam_h, u)), ykd::mul(cam_v, v)), cam_o);
  o = cam_o;
  if (lens) {  // thin-lens offset
    const double rx = px * cam.lens_radius, ry = py * cam.lens_radius;
    const v3 off = ykd::add(ykd::mul(ld3(cam.lens_u), rx), ykd::mul(ld3(cam.lens_v), ry));
    o = ykd::add(o, off);
    d = ykd::sub(d, off);
  }
}
// the same in float (camera<float>, the host-rounded camera CamF; (x + U01) / W a float division)
__device__ __forceinline__ void camera_ray_f32(const CamF& cam, uint32_t H, uint32_t x, uint32_t y, float uc,
                                               float vc, bool lens, float px, float py, ykf::v3& o, ykf::v3& d) {
  const float u = ((float)x + uc) / cam.w;
  const float v = ((float)(H - y - 1) + vc) / cam.h;
  const ykf::v3 cam_o = ykf::off(cam.origin), cam_llc = ykf::off(cam.llc);
  const ykf::v3 cam_h = ykf::off(cam.horizontal), cam_v = ykf::off(cam.vertical);
  d = ykf::sub(ykf::add(ykf::add(cam_llc, ykf::mul(cam_h, u)), ykf::mul(cam_v, v)), cam_o);
  o = cam_o;
  if (lens) {
    const float rx = px * cam.lens_radius, ry = py * cam.lens_radius;
    const ykf::v3 off = ykf::add(ykf::mul(ykf::off(cam.lens_u), rx), ykf::mul(ykf::off(cam.lens_v), ry));
    o = ykf::add(o, off);
    d = ykf::sub(d, off);
  }
}

// A sample's start, precomputed by yk_mt_warmup for the mt19937 kernels: the camera ray of the
// sample (after the jitter canonicals and the thin-lens rejection loop) and the lazy cursors
// after those draws (x_j, x_{j+1}, x_{j+397}, j).  j == kNoStart: the lens loop would have
// reached the scratch engine's words (never seen: ~55 rejections), and the render kernel starts
// that sample itself.  FP64: 64 bytes (four 16-byte loads); FP32: 48.
struct alignas(16) StartRec {
  double ox, oy, oz, dx, dy, dz;
  uint32_t a0, a1, b, j;
};
static_assert(sizeof(StartRec) == 64, "StartRec layout");
struct alignas(16) StartRecF {
  float ox, oy, oz, dx, dy, dz;
  uint32_t pad0, pad1;
  uint32_t a0, a1, b, j;
};
static_assert(sizeof(StartRecF) == 48, "StartRecF layout");
constexpr uint32_t kNoStart = 0xffffffffu;
// j == kPadSlot: the slot is an empty slot of an edge block (kNoPixel in the processing order), so
// the render tells it from its StartRec alone and reads the order only for a start it makes itself
constexpr uint32_t kPadSlot = 0xfffffffeu;
constexpr uint32_t kPadX = 0xffffffffu;  // (the warm-up's column of such a slot)

// Seed walk and start of every sample of a launch, fully coherent, one sample per thread
// (grid-stride): the 397-step walk, then the start's draws with the lazy cursors (yk_device.hpp)
// and the camera ray, which thereby leave the divergent render loop.  kLens: the camera has a
// lens (the rejection loop is compiled only then: its registers cost co-resident waves); kF32:
// the FP32 kernel's start (one-word float canonicals, ykf::canonical; camera<float>).  The walk
// is ~400 dependent steps per sample (8.9e12 steps/s on the whole GPU, tools/walkbench.hip: 47 ms
// of a 512-spp frame if it ran alone), so these waves live on the render's idle issue cycles at
// lower priority.  One sample per thread (two or four interleaved: 204.6 -> 211.2 / 215.5 ms,
// 512-spp A/B): 32 VGPRs with a lens, so four of these waves fit beside the three 128-VGPR
// render waves of a SIMD (a record of the draws instead of the ray: 20 VGPRs and five waves,
// 0.5% slower, r03ab).
struct WarmArgs {
  uint32_t W, spp, seed0, row_begin, row_stride, s0, npix_slots, seed_mode, band_log2;
  uint32_t Wt, col_begin, col_stride, col_band;  // the tile's columns (as KernelArgs)
  uint32_t nps_m, nps_sh, w_m, w_sh;  // fdiv magic numbers of npix_slots and the tile width Wt
  uint32_t lens, H;                   // the camera has a lens (lens_radius > 0); image height
  uint64_t seed_key;
  yk_camera cam;
  CamF camf;
  double w_d, h_d, inv_w, inv_h;      // as in KernelArgs
  const uint32_t* order;
  uint64_t n;  // sample slots in the launch
  void* out;
  uint32_t* counter;  // the launch's sample-slot counter: cleared here (the render waits for this kernel)
  uint4* retry;         // yk_mt_warmup_defer: the lens retries, retry_cap records of 48 B per wave
  uint32_t retry_cap, retry_pad;
};

// Thin-lens retries after the walks (yk_mt_warmup_defer): a sample whose first random_in_unit_disk candidate is
// rejected leaves its engine state (slot, seed, cursors, jitter canonicals) in its wave's ring and
// the wave draws the further candidates for 64 such samples at a time once its grid-stride walks
// are done, so no wave runs the rejection loop for its unluckiest lane (3.6 candidate draws per
// wave-sample against 1.27 per sample).  A sample that finds its wave's ring full is handed to the
// render as a start it makes itself (kNoStart), as a lens loop that runs out of lazy words is.
// records per wave: the rejections of the wave's slots (p = 1 - pi/4) + 6 sigma + a batch
inline uint32_t retry_cap_for(uint64_t slots_per_wave) {
  const double m = 0.2146 * (double)slots_per_wave, sd = std::sqrt(m * 0.7854);
  return ((uint32_t)(m + 6.0 * sd) + 64u + 63u) & ~63u;
}
__device__ __forceinline__ void retry_put(uint4* r, uint32_t i, const ykd::MtLane& g, double uc, double vc) {
  r[0] = make_uint4(i, g.seed, g.a0, g.a1);
  r[1] = make_uint4(g.b, g.j, 0u, 0u);
  *(double2*)(r + 2) = make_double2(uc, vc);
}
// (agent-scope relaxed loads: global_load ... sc1, past this CU's L1 — another lane of the wave
// wrote the record, and the ring's positions are rewritten)
__device__ __forceinline__ uint64_t ld_l2(const uint4* r, int k) {
  return __hip_atomic_load((const uint64_t*)r + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint32_t retry_get(const uint4* r, ykd::MtLane& g, double& uc, double& vc) {
  const uint64_t w0 = ld_l2(r, 0), w1 = ld_l2(r, 1), w2 = ld_l2(r, 2);
  g.state = nullptr;
  g.seed = (uint32_t)(w0 >> 32);
  g.a0 = (uint32_t)w1;
  g.a1 = (uint32_t)(w1 >> 32);
  g.b = (uint32_t)w2;
  g.j = (uint32_t)(w2 >> 32);
  uc = __longlong_as_double((long long)ld_l2(r, 4));
  vc = __longlong_as_double((long long)ld_l2(r, 5));
  return (uint32_t)w0;
}

// kIlp: the seed walks of kIlp slots interleaved per lane (i, i + stride, ...; the walk is a
// chain of dependent instructions), their starts then one after the other
template <bool kLens, bool kF32, bool kDefer, uint32_t kIlp>
__device__ __forceinline__ void mt_warmup_body(const WarmArgs& wa) {
  constexpr uint32_t kWarmBlock = 256;  // (every warm-up launches 256-thread blocks)
  // (32-bit indices: a launch keeps its slots below 2^31 and the grid below 2^21 threads)
  const uint32_t n = (uint32_t)wa.n;
  const uint32_t stride = gridDim.x * kWarmBlock;
  if (blockIdx.x == 0 && threadIdx.x == 0) *wa.counter = 0u;
  static_assert(!kDefer || (kLens && !kF32), "the deferred lens loop is the FP64 lens warm-up's");
  // kDefer: this wave's ring and how many records it holds (every lane of the wave enqueues in
  // step: a lane that has left the loop never holds the count alone, lane 0 leaves last)
  uint4* const ring =
      kDefer ? wa.retry + (size_t)__builtin_amdgcn_readfirstlane((blockIdx.x * kWarmBlock + threadIdx.x) >> 6) *
                              wa.retry_cap * 3
             : nullptr;
  uint32_t rcount = 0;
  // slot i's pixel (xx, y) and seed; an empty slot gets column kPadX (its record is marked)
  auto slot_seed = [&](uint32_t i, uint32_t& xx, uint32_t& y) -> uint32_t {
    const uint32_t sl = fdiv(i, wa.nps_m, wa.nps_sh), pp = i - sl * wa.npix_slots;
    const uint32_t q = wa.order[pp];
    const uint32_t pix = q == kNoPixel ? 0u : q;
    const uint32_t tr = fdiv(pix, wa.w_m, wa.w_sh);
    xx = tile_col_x(wa.col_begin, wa.col_stride, wa.col_band, pix - tr * wa.Wt);
    y = tile_row_y(wa.row_begin, wa.row_stride, wa.band_log2, tr);
    const uint32_t seed = ykd::sample_seed(wa.seed_mode, wa.seed_key, wa.seed0, y, xx, wa.W, wa.spp, wa.s0 + sl);
    xx = q == kNoPixel ? kPadX : xx;
    return seed;
  };
  // the start of slot i after its walk: draws, lens, camera ray, record
  auto start_slot = [&](uint32_t i, uint32_t xx, uint32_t y, uint32_t seed, uint32_t x397) {
    ykd::MtLane g;
    g.state = nullptr;
    ykd::mt_start_from(g, seed, x397);
    bool failed = false;  // the lens loop would reach the scratch engine's words
    if constexpr (kF32) {
      const float uc = ykf::canonical<true>(g);  // source.cpp:162 with T = float
      const float vc = ykf::canonical<true>(g);  // source.cpp:163
      float px = 0.0f, py = 0.0f;
      if (kLens) {
        for (;;) {  // thin-lens extension: random_in_unit_disk by rejection, x then y
          if (!ykd::rng_lazy_ok(g, 2)) {
            failed = true;
            break;
          }
          px = ykf::uniform_of(ykf::canonical<true>(g), -1.0f, 1.0f);
          py = ykf::uniform_of(ykf::canonical<true>(g), -1.0f, 1.0f);
          if (px * px + py * py < 1.0f) break;
        }
      }
      ykf::v3 o, d;
      camera_ray_f32(wa.camf, wa.H, xx, y, uc, vc, kLens, px, py, o, d);
      uint4* const out = (uint4*)wa.out + 3 * (size_t)i;
      *(float4*)out = make_float4(o.x, o.y, o.z, d.x);
      *(float4*)(out + 1) = make_float4(d.y, d.z, 0.0f, 0.0f);
      out[2] = make_uint4(g.a0, g.a1, g.b, xx == kPadX ? kPadSlot : failed ? kNoStart : g.j);
    } else {
      const double uc = ykd::canonical<true>(g);  // source.cpp:162
      const double vc = ykd::canonical<true>(g);  // source.cpp:163
      double px = 0.0, py = 0.0;
      if constexpr (kDefer) {
        // the first candidate in line; a rejected sample goes to the ring while it has room
        bool again = false;
        if (!ykd::rng_lazy_ok(g, 4)) {
          failed = true;
        } else {
          px = ykd::uniform<true>(g, -1, 1);
          py = ykd::uniform<true>(g, -1, 1);
          again = !(px * px + py * py < 1.0);
        }
        const unsigned long long m = __ballot(again);
        const uint32_t nq = (uint32_t)__popcll(m);
        const bool room = rcount + nq <= wa.retry_cap;
        if (room) {
          if (again) {
            const uint32_t pos = rcount + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            retry_put(ring + 3 * pos, i, g, uc, vc);
          }
          rcount += nq;
          if (again) return;
        } else if (again) {
          failed = true;  // (the ring is full: the render kernel starts this sample itself)
        }
      } else if (kLens) {
        for (;;) {
          if (!ykd::rng_lazy_ok(g, 4)) {
            failed = true;
            break;
          }
          px = ykd::uniform<true>(g, -1, 1);
          py = ykd::uniform<true>(g, -1, 1);
          if (px * px + py * py < 1.0) break;
        }
      }
      v3 o, d;
      camera_ray(wa.cam, wa.w_d, wa.inv_w, wa.h_d, wa.inv_h, wa.H, xx, y, uc, vc, kLens, px, py, o, d);
      uint4* const out = (uint4*)wa.out + 4 * (size_t)i;
      *(double2*)out = make_double2(o.x, o.y);
      *(double2*)(out + 1) = make_double2(o.z, d.x);
      *(double2*)(out + 2) = make_double2(d.y, d.z);
      out[3] = make_uint4(g.a0, g.a1, g.b, xx == kPadX ? kPadSlot : failed ? kNoStart : g.j);
    }
  };
  if constexpr (kIlp > 1) {
    for (uint32_t i = blockIdx.x * kWarmBlock + threadIdx.x; i < n; i += kIlp * stride) {
      uint32_t xx, y, x[kIlp];
#pragma unroll
      for (uint32_t k = kIlp - 1; k > 0; --k) {
        const uint32_t ik = i + k * stride;
        x[k] = slot_seed(ik < n ? ik : i, xx, y);
      }
      const uint32_t seed = slot_seed(i, xx, y);
      x[0] = seed;
      ykd::mt_walk397xn<kIlp>(x);
      start_slot(i, xx, y, seed, x[0]);
#pragma unroll
      for (uint32_t k = 1; k < kIlp; ++k) {
        const uint32_t ik = i + k * stride;
        if (ik < n) {
          const uint32_t sk = slot_seed(ik, xx, y);
          start_slot(ik, xx, y, sk, x[k]);
        }
      }
    }
  } else {
    for (uint32_t i = blockIdx.x * kWarmBlock + threadIdx.x; i < n; i += stride) {
      uint32_t xx, y;
      const uint32_t seed = slot_seed(i, xx, y);
      uint32_t x[1] = {seed};
      ykd::mt_walk397xn<1>(x);
#ifdef YK_WALK_SENS
      // (sensitivity probe, never in the product: YK_WALK_SENS more walks of a perturbed seed, their
      // result folded in as a no-op the compiler cannot prove)
      for (int r_ = 0; r_ < YK_WALK_SENS; ++r_) {
        uint32_t z[1] = {seed ^ (0x9e3779b9u + (uint32_t)r_)};
        ykd::mt_walk397xn<1>(z);
        x[0] ^= (z[0] == 0x12345678u && seed == 0x9abcdef0u) ? 1u : 0u;
      }
#endif
      start_slot(i, xx, y, seed, x[0]);
    }
  }
  if constexpr (kDefer) {
    // the ring: one more candidate for up to 64 records per trip, the rejected re-queued at its end
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t head = 0, cnt = __builtin_amdgcn_readfirstlane(rcount);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the records are in L2
    while (cnt > 0u) {
      const uint32_t take = min(cnt, 64u);
      const bool act = lane < take;
      ykd::MtLane g;
      double uc = 0, vc = 0, px = 0, py = 0;
      uint32_t i = 0;
      bool again = false, failed = false;
      if (act) {
        uint32_t pos = head + lane;
        pos = pos >= wa.retry_cap ? pos - wa.retry_cap : pos;
        i = retry_get(ring + 3 * pos, g, uc, vc);
        if (!ykd::rng_lazy_ok(g, 4)) {
          failed = true;
        } else {
          px = ykd::uniform<true>(g, -1, 1);
          py = ykd::uniform<true>(g, -1, 1);
          again = !(px * px + py * py < 1.0);
        }
      }
      head += take;
      head = head >= wa.retry_cap ? head - wa.retry_cap : head;
      cnt -= take;
      const unsigned long long m = __ballot(again);
      if (again) {
        uint32_t pos = head + cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        pos = pos >= wa.retry_cap ? pos - wa.retry_cap : pos;
        retry_put(ring + 3 * pos, i, g, uc, vc);
      }
      cnt += (uint32_t)__popcll(m);
      if (act && !again) {
        const uint32_t sl = fdiv(i, wa.nps_m, wa.nps_sh), pp = i - sl * wa.npix_slots;
        const uint32_t q = wa.order[pp];
        const uint32_t pix = q == kNoPixel ? 0u : q;
        const uint32_t tr = fdiv(pix, wa.w_m, wa.w_sh);
        const uint32_t xx = tile_col_x(wa.col_begin, wa.col_stride, wa.col_band, pix - tr * wa.Wt);
        const uint32_t y = tile_row_y(wa.row_begin, wa.row_stride, wa.band_log2, tr);
        uint4* const out = (uint4*)wa.out + 4 * (size_t)i;
        out[3] = make_uint4(g.a0, g.a1, g.b, q == kNoPixel ? kPadSlot : failed ? kNoStart : g.j);
        v3 o, d;
        camera_ray(wa.cam, wa.w_d, wa.inv_w, wa.h_d, wa.inv_h, wa.H, xx, y, uc, vc, kLens, px, py, o, d);
        *(double2*)out = make_double2(o.x, o.y);
        *(double2*)(out + 1) = make_double2(o.z, d.x);
        *(double2*)(out + 2) = make_double2(d.y, d.z);
      }
      if (cnt > 0u) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  }
}

// Walks per lane: the deferred FP64 lens warm-up (the headline frame's) walks four slots at once at
// 48 VGPRs, so two of its waves share a SIMD with the three render waves (eight walk chains per
// SIMD instead of four: bench -0.9%, r05_ab/walk/); the other warm-ups walk one
#ifndef YK_WALK_ILP
#define YK_WALK_ILP 4
#endif
#ifndef YK_WALK_ILP_INLINE
#define YK_WALK_ILP_INLINE 1
#endif
constexpr uint32_t kWalkIlp = YK_WALK_ILP, kWalkIlpInline = YK_WALK_ILP_INLINE;
template <bool kLens, bool kF32>
__global__ __launch_bounds__(256) void yk_mt_warmup(WarmArgs wa) {
  mt_warmup_body<kLens, kF32, false, kWalkIlpInline>(wa);
}
// the FP64 lens warm-up with its retries deferred, at 48 VGPRs: two of its waves beside the three
// 128-VGPR render waves of a SIMD (the attribute counts gfx950's unified register file: twice)
#ifndef YK_DEFER_VGPRS
#define YK_DEFER_VGPRS 48
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_vgpr(YK_DEFER_VGPRS / 2))) void yk_mt_warmup_defer(WarmArgs wa) {
  mt_warmup_body<true, false, true, kWalkIlp>(wa);
}

// kSceneInLds: the BVH nodes, the leaf-ordered sphere geometry and the leaf→tuple ids are copied
// into LDS by each workgroup once (33 KB for the 485-sphere scene), so a node visit is four
// ds_read_b128 instead of four dependent L2 round trips.  Larger scenes read them from global.

// A sample's colour record: r, g, b as one aligned 32-byte record per sample slot (one 16-byte
// and one 8-byte store, the whole record in one 32-byte sector), in a colour buffer of the launch.
// yk_reduce_samples reads the records of consecutive slots, coalesced.  (Round 4 tried writing
// the colour over the slot's own StartRec instead — no colour buffer at all — and the frame got
// 3% slower: 174.1 -> 179.5 ms, profiles/r04_ab/; the reduce then reads 24 of every 64 bytes.)
constexpr size_t kColStride = 4;
__device__ __forceinline__ void colour_store(double* col, uint32_t slot, double r, double g, double b) {
  double* rec = col + (size_t)slot * kColStride;
  *(double2*)rec = make_double2(r, g);
  rec[2] = b;
}

// Ordered sum of a launch's sample colours per pixel: pixel_color of source.cpp:137-167 is the
// left fold ((0 + c_0) + c_1) + ... in sample order, continued across launches through acc; after
// the last launch, to_color3b (source.cpp:73-83): /spp, math::sqrt, clamp [0, .999], *256,
// truncate.  One thread per processing slot, coalesced over the SoA colours.
struct ReduceArgs {
  const double* col;  // col[(s_local * npix_slots + p) * kColStride + c]
  double* acc;        // running sums, acc[c * npix_slots + p]
  const uint32_t* order;
  uint8_t* rgb;
  double* sums;
  uint32_t npix_slots, nsl, ks, spp;
  uint32_t first, last, pad0, pad1;
};
__device__ __forceinline__ void reduce_slot(const ReduceArgs& ra, uint32_t p) {
  const uint32_t q = ra.order[p];
  if (q == kNoPixel) return;
  double a[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) a[c] = ra.first ? 0.0 : ra.acc[(size_t)c * ra.npix_slots + p];
  for (uint32_t k = 0; k < ra.ks; ++k) {
    const size_t i = (size_t)k * ra.npix_slots + p;
#pragma unroll
    for (int c = 0; c < 3; ++c) a[c] = a[c] + ra.col[i * kColStride + c];
  }
  if (!ra.last) {
#pragma unroll
    for (int c = 0; c < 3; ++c) ra.acc[(size_t)c * ra.npix_slots + p] = a[c];
    return;
  }
  const size_t o3 = (size_t)q * 3;
  const double spp = (double)ra.spp;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    if (ra.sums) ra.sums[o3 + c] = a[c];
    double v = ykd::nsqrt(a[c] / spp);
    v = (v < 0.0) ? 0.0 : (0.999 < v) ? 0.999 : v;
    ra.rgb[o3 + c] = (uint8_t)(uint32_t)(v * 256);
  }
}
__global__ __launch_bounds__(256) void yk_reduce_samples(ReduceArgs ra) {
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < ra.npix_slots; p += gridDim.x * blockDim.x)
    reduce_slot(ra, p);
}

// The refined reciprocal of every radius, by the same instructions the division sequence uses
// (rcp_refined), so the hit normal's (p - c) / radius reuses it (divs_fast_r: bit-identical to
// divs_fast).  Run once per set_scene.
__global__ void yk_mat_prep(SphereMat* m, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    m[i].inv_r = ykd::rcp_refined(m[i].radius);
    m[i].inv_rf = ykf::rcp_refined((float)m[i].radius);
  }
}

// ykgpu_math_div: the renderer's vector / scalar division (divs_fast) on a buffer (diagnostic).
__global__ __launch_bounds__(256) void yk_math_div(const double* num3, const double* den, double* out3,
                                                  uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ykd::v3 q = ykd::divs_fast({num3[3 * i], num3[3 * i + 1], num3[3 * i + 2]}, den[i]);
  out3[3 * i] = q.x;
  out3[3 * i + 1] = q.y;
  out3[3 * i + 2] = q.z;
}

// ykgpu_math_div_f32: the FP32 kernel's vector / scalar division (ykf::divs_fast) on a buffer.
__global__ __launch_bounds__(256) void yk_math_div_f32(const float* num3, const float* den, float* out3, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ykf::v3 q = ykf::divs_fast({num3[3 * i], num3[3 * i + 1], num3[3 * i + 2]}, den[i]);
  out3[3 * i] = q.x;
  out3[3 * i + 1] = q.y;
  out3[3 * i + 2] = q.z;
}

// ykgpu_math_sqrt: the device's math::sqrt on a buffer (diagnostic entry point).
__global__ __launch_bounds__(256) void yk_math_sqrt(const double* in, double* out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = ykd::nsqrt(in[i]);
}

// Refill of the persistent kernels: lanes without a path take the next sample slots from the
// wave's reserve, one atomic per kClaim slots.  Every lane runs it, so the reserve (res_base,
// res_left) stays wave-uniform.  (A pixel is not a lane's unit of work: the samples of a pixel
// are independent, only their SUM is ordered, and yk_reduce_samples does that.)  Returns true
// when this lane has no path and the launch has no slots left: the lane exits.
// The per-sample engine of a kernel instance (YK_RNG_*): lane set-up.
__device__ __forceinline__ void rng_init(ykd::MtLane& g, const KernelArgs& ka, uint32_t gid) {
  g.state = ka.mt_scratch + (size_t)gid * ykd::kMtN;
  g.a0 = g.a1 = g.b = g.j = g.seed = 0;
}
__device__ __forceinline__ void rng_init(ykd::X128Lane& g, const KernelArgs&, uint32_t) { g.x = g.y = g.z = g.w = g.n = 0; }

// A sample's engine from its seed alone (xor128, and an mt19937 start no StartRec serves):
// mt19937 walks its 397 seeding steps here
__device__ __forceinline__ void rng_start_full(ykd::MtLane& g, uint32_t seed) { ykd::mt_start(g, seed); }
__device__ __forceinline__ void rng_start_full(ykd::X128Lane& g, uint32_t seed) { ykd::x128_start(g, seed); }

__device__ __forceinline__ bool claim_slots(const KernelArgs& ka, bool in_path, uint32_t lane, uint32_t& slot,
                                            uint32_t& res_base, uint32_t& res_left) {
  const unsigned long long m = __ballot(!in_path);
  if (m) {
    const uint32_t need = (uint32_t)__popcll(m);
    uint32_t fresh = 0, csize = kClaim;
    if (res_left < need) {
      if (kClaimTail) {
        // res_base + res_left: where the counter stood after this wave's last claim
        const uint32_t seen = res_base + res_left;
#if YK_CLAIM_ARGS
        const uint32_t tail = ka.claim_tail;  // (the host's: no dispatch-packet load, no vmcnt wait)
#else
        const uint32_t tail = gridDim.x * (blockDim.x >> 6) * kClaim * kClaimTailFactor;
#endif
        if (seen >= ka.nsl || ka.nsl - seen < tail) csize = kClaimTail;
      }
      const int leader = __ffsll((long long)m) - 1;
      if ((int)lane == leader) fresh = atomicAdd(ka.pixel_counter, csize);
#if YK_CLAIM_ARGS
      fresh = __builtin_amdgcn_readlane(fresh, leader);  // (the leader is wave-uniform)
#else
      fresh = __shfl(fresh, leader);
#endif
    }
    if (!in_path) {
      const uint32_t r = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      slot = r < res_left ? res_base + r : fresh + (r - res_left);
    }
    if (res_left < need) {
      res_base = fresh + (need - res_left);
      res_left = csize - (need - res_left);
    } else {
      res_base += need;
      res_left -= need;
    }
  }
  return !in_path && slot >= ka.nsl;
}

using RenderKernel = void (*)(KernelArgs);

// YK_SPLIT (Makefile): 0 — every kernel in this translation unit (the A/B variants of
// tools/build_def_variant.sh); 1 — the library's main unit, without the FP32 render kernel; 2 —
// the FP32 render kernel alone, compiled under LLVM's max-ilp scheduler (FP32 512 spp: -1.3%;
// the same scheduler costs the FP64 kernel +1.5%)
#ifndef YK_SPLIT
#define YK_SPLIT 0
#endif
#if YK_SPLIT != 2
// kCount: the work counters of YK_FLAG_COUNT_WORK (an instance of its own, so the production
// instance carries neither their registers nor their adds)
// kMode bit 0: the work counters; bit 1: YK_SEED_RANDOM_DEVICE seeding (an instance of its own:
// the hash's 64-bit arithmetic and two more kernel arguments cost the counter-seeded production
// instance 0.6% through SGPR spills); bit 2: the yk::xor128 engine (YK_RNG_XOR128)
template <bool kSceneInLds, int kMode>
__device__ __forceinline__ void render_body(KernelArgs ka) {
  constexpr int kBlk = mode_block<kMode>();
  constexpr bool kCount = (kMode & 1) != 0;
  constexpr bool kRandomSeed = (kMode & 2) != 0;
  using Gen = typename std::conditional<(kMode & 4) != 0, ykd::X128Lane, ykd::MtLane>::type;
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const char* __restrict__ nodes = (const char*)ka.nodes;
  const SphereGeo* __restrict__ leaf_geo = ka.leaf_geo;
  const uint32_t* __restrict__ leaf_ids = ka.leaf_ids;
  const SphereGeo* __restrict__ geo = ka.geo;  // tuple order: candidates' roots, hit records
  const SphereMat* __restrict__ mat = ka.mat;  // shading, attenuation unwind
  if (kSceneInLds) {
    // the BVH, its leaf geometry and ids, and (tuple order) the geometry and materials
    const uint4* src[5] = {(const uint4*)ka.nodes, (const uint4*)ka.leaf_geo, (const uint4*)ka.leaf_ids,
                           (const uint4*)ka.geo, (const uint4*)ka.mat};
    const uint32_t off[5] = {0u, ka.lds_geo_off, ka.lds_ids_off, ka.lds_tgeo_off, ka.lds_mat_off};
    const uint32_t n16[5] = {(ka.n_nodes * (uint32_t)sizeof(DevNode) + 15u) / 16u, ka.nspheres * 2u,
                             (ka.nspheres + 3u) / 4u, ka.nspheres * 2u, ka.nspheres * 4u};
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      uint4* dst = (uint4*)(smem + off[k]);
      for (uint32_t i = threadIdx.x; i < n16[k]; i += kBlk) dst[i] = src[k][i];
    }
    __syncthreads();
    nodes = smem;
#if YK_NODE_BF
    // the child-code reads address the LDS copy from 0: the dynamic region must start there
    if ((uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)smem != 0u) __builtin_trap();
#endif
    leaf_geo = (const SphereGeo*)(smem + ka.lds_geo_off);
    leaf_ids = (const uint32_t*)(smem + ka.lds_ids_off);
    geo = (const SphereGeo*)(smem + ka.lds_tgeo_off);
    mat = (const SphereMat*)(smem + ka.lds_mat_off);
  }
  int32_t* const stk = (int32_t*)(smem + ka.lds_stack_off) + threadIdx.x;  // [sp * kBlk]
  // YK_FLAG_ONE_LANE (counting instance only): lanes 1..63 leave here, after the block's last
  // barrier, so every wave-instruction below is one lane's (the profiler's per-wave FP64 counters
  // then count that lane's executed operations exactly: DESIGN.md §5)
  if (kCount && (ka.flags & kFlagOneLane) && lane != 0) return;
#if YK_NODE_BF
  stk[0] = ykbvh::kEmptyLeaf;  // the sentinel below every traversal's entries
#endif
#if YK_RENDER_PRIO
  // the warm-up waves sharing the SIMDs (priority 0) get only the issue slots the render leaves
  __builtin_amdgcn_s_setprio(YK_RENDER_PRIO);
#endif
  YK_CLOCK_BEGIN(ka);
  YK_WAVE_STAMP(ka, 0);

  Gen g;
  rng_init(g, ka, gid);
  uint16_t* const id_spill = ka.id_scratch + (size_t)gid * ka.id_stride;

  uint32_t n_seg = 0, n_test = 0, n_sqrt = 0, n_fb = 0, n_node = 0, n_lin = 0, n_ncall = 0, n_nit = 0;
  uint32_t n_dpos = 0;  // leaf tests with disc >= 0 (their root bounds are computed)
  uint32_t n_lamb = 0, n_metal = 0, n_fuzz = 0, n_diel = 0;  // hits shaded per material kind
  // engine words drawn (the warm-up's start words among them) and scratch-engine twists
  uint32_t n_words = 0, n_swords = 0, n_twist = 0;

  YK_STAMPS_BEGIN(ka.counters, lane);
  uint32_t slot = 0, depth = 0, nstk = 0;
  uint32_t st0 = 0, st1 = 0, st2 = 0, st3 = 0;  // newest attenuation id in st0's low half
  v3 o = {0, 0, 0}, d = {0, 0, 0};
  bool in_path = false;
  // wave-level reserve of claimed sample slots (identical in every lane of the wave)
  uint32_t res_base = 0, res_left = 0;

  for (;;) {
    // ---- refill (claim_slots): lanes without a path take the next sample slots
    if (claim_slots(ka, in_path, lane, slot, res_base, res_left)) {
      YK_STAMPS_EXHAUSTED(ka.counters);
      break;
    }
    YK_STAMP(0);

    // ---- start sample s of the pixel: seed, jitter, camera ray (source.cpp:154-165) ------
    bool start = !in_path;
    // mt19937: the slot's StartRec, its four loads issued together and waited for once (every
    // slot of the launch, empty ones included, has a record, so the read is in bounds); it says
    // whether the slot is empty (kPadSlot) and holds the whole start, so neither the processing
    // order nor the pixel's seed is read here — the scratch engine recovers the seed from its
    // cursor (mt_slow).  xor128: the slot's pixel
    uint4 rq0 = {0, 0, 0, 0}, rq1 = {0, 0, 0, 0}, rq2 = {0, 0, 0, 0}, rq3 = {0, 0, 0, 0};
    uint32_t qpix = 0;
    if (start) {
      if constexpr (std::is_same<Gen, ykd::MtLane>::value) {
        const uint4* rp = (const uint4*)ka.start + 4u * slot;
        rq0 = rp[0];
        rq1 = rp[1];
        rq2 = rp[2];
        rq3 = rp[3];
        asm volatile("" ::"v"(rq0.x), "v"(rq0.y), "v"(rq0.z), "v"(rq0.w), "v"(rq1.x), "v"(rq1.y),
                     "v"(rq1.z), "v"(rq1.w), "v"(rq2.x), "v"(rq2.y), "v"(rq2.z), "v"(rq2.w), "v"(rq3.x),
                     "v"(rq3.y), "v"(rq3.z), "v"(rq3.w));
        start = rq3.w != kPadSlot;  // an empty slot of an edge block: take another next trip
      } else {
        const uint32_t sl = fdiv(slot, ka.nps_m, ka.nps_sh);
        qpix = ka.order[slot - sl * ka.npix_slots];
        start = qpix != kNoPixel;
      }
    }
    if (start) {
      // The start — the jitter canonicals, the lens point and the camera ray — and the engine
      // after its draws: precomputed for mt19937 by yk_mt_warmup (StartRec), so the divergent
      // loop only loads them; xor128, and the (never seen) record the warm-up could not
      // complete, start here
      bool pre = false;
      if constexpr (std::is_same<Gen, ykd::MtLane>::value) {
        StartRec r;  // (loaded above)
        __builtin_memcpy((char*)&r, &rq0, 16);
        __builtin_memcpy((char*)&r + 16, &rq1, 16);
        __builtin_memcpy((char*)&r + 32, &rq2, 16);
        __builtin_memcpy((char*)&r + 48, &rq3, 16);
        pre = r.j != kNoStart;
        if (pre) {
          if (kCount) n_swords += r.j;
          g.a0 = r.a0;
          g.a1 = r.a1;
          g.b = r.b;
          g.j = r.j;
          o = v3{r.ox, r.oy, r.oz};
          d = v3{r.dx, r.dy, r.dz};
        }
      }
      if (!pre) {
        // the pixel and its seed (uint32 wrap, source.cpp:154-158)
        const uint32_t sl = fdiv(slot, ka.nps_m, ka.nps_sh);
        if constexpr (std::is_same<Gen, ykd::MtLane>::value) qpix = ka.order[slot - sl * ka.npix_slots];
        const uint32_t s = ka.s0 + sl;
        const uint32_t tr = fdiv(qpix, ka.w_m, ka.w_sh);
        const uint32_t x = tile_col_x(ka.col_begin, ka.col_stride, ka.col_band, qpix - tr * ka.Wt);
        const uint32_t y = tile_row_y(ka.row_begin, ka.row_stride, ka.band_log2, tr);
        const uint32_t seed = ykd::sample_seed(kRandomSeed ? 1u : 0u, ka.seed_key, ka.seed0, y, x, ka.W, ka.spp, s);
        const bool lens = ka.cam.lens_radius > 0;
        rng_start_full(g, seed);
        const double uc = ykd::canonical<true>(g);  // (a fresh engine: its first words never need the scratch engine)
        const double vc = ykd::canonical<true>(g);
        double px = 0, py = 0;
        if (lens) {  // thin-lens extension: random_in_unit_disk by rejection
          do {
            px = ykd::uniform(g, -1, 1);
            py = ykd::uniform(g, -1, 1);
          } while (!(px * px + py * py < 1.0));
        }
        camera_ray(ka.cam, ka.w_d, ka.inv_w, ka.h_d, ka.inv_h, ka.H, x, y, uc, vc, lens, px, py, o, d);
      }
      depth = ka.max_depth;
      nstk = 0;
      in_path = true;
    }
    YK_STAMP(1);
    // ray_color prints its ray before the depth test (raytracer.hpp:21-25)
    if (kCount && (ka.flags & kFlagTrace) && in_path) trace_ray(ka, slot, ka.max_depth - depth, o, d);

    // ---- one segment of ray_color (raytracer.hpp:19-37) ----------------------------------
    // (a) closest hit: hittable_list::hit_impl (hittable_list.hpp:32-58) over
    //     sphere::hit_impl (sphere.hpp:25-48): tuple order, t_max shrinking to the last
    //     accepted root, so the closest hit wins and an exact tie goes to the later sphere.
    // depth == 0 → black (raytracer.hpp:23); lanes without a path (empty slot) sit this out
    const bool alive = in_path && depth != 0;
    Hit hit{INFINITY, -1, 0, 0, 0, 0};
    if (alive) {
      ++n_seg;
      const double a = ykd::len2(d);
      const double onorm = fmax(fabs(o.x), fmax(fabs(o.y), fabs(o.z)));
      bool linear = (ka.flags & kFlagLinearScan) || !(a > 0 && a < INFINITY) ||
                    !(onorm <= ka.origin_bound);
      if (!linear) {
        // BVH traversal: cull conservatively, keep every sphere whose exact root could be
        // the minimum.  Slab distances as one FMA each,
        // t = lo*(1/d) - o*(1/d): error relative 2^-22 plus an origin perturbation of
        // 2^-23|o| (< delta/4), inside the culling contract of yk_bvh.hpp.  This is culling
        // arithmetic only, so explicit FMAs are fine here.
        // 1/d from v_rcp_f32 (1 ulp): with d's rounding to float and the FMA's rounding the
        // slab distances stay within the 2^-22 relative error the culling contract assumes
        // (2^-24 + 2^-23 + 2^-24).  Components outside [1e-30, 1e30] (never seen) take the
        // correctly rounded division for the whole wave.
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
        // this ray's (near x4, far x4) plane quads inside a WideNode (yk_bvh.hpp), as base
        // pointers: a visit then costs one address add per axis
        const char* const px = nodes + (ix < 0.0f ? 16u : 0u);
        const char* const py = nodes + 48u + (iy < 0.0f ? 16u : 0u);
        const char* const pz = nodes + 96u + (iz < 0.0f ? 16u : 0u);
        // Conservative interval test without per-visit relaxation: far distances
        // come out of the FMA already scaled by c = 1 + 2^-17 (scaled 1/d and o/d), near
        // distances are compared unscaled against tmin_lo = t_min (1 - 2^-17) and against
        // ustar_f (U* (1 + 2^-18)).  A box passes iff
        //   max(tn, tmin_lo) <= min(tf * c, ustar_f),
        // which holds whenever the former test with both distances relaxed by 2^-20 held.
        constexpr float kFar = 1.0f + 0x1p-17f;
        // scaled far terms: ONE rounding of the origin product, as for the near terms, so the
        // origin perturbation stays within delta/4 (yk_bvh.hpp); the rounding of ix*c is a
        // relative error inside the 2^-17 margin
        const float ixs = ix * kFar, iys = iy * kFar, izs = iz * kFar;
        const float ox_f = (float)o.x, oy_f = (float)o.y, oz_f = (float)o.z;
        const float tmin_lo = __double2float_rd(ka.t_min) * (1.0f - 0x1p-17f);
#if YK_SLAB_PAIRS_F64 && YK_NEAR_CLAMP
        // Distances measured from tmin_lo and scaled by kClampScale = 2^-24: per
        // axis (s/d, s(-o/d - tmin_lo)) (near) and (sc/d, s(-oc/d - tmin_lo)) (far).  The near
        // FMAs clamp to [0, 1], which IS the max with tmin_lo (distances below 2^24 + tmin_lo
        // never reach the clamp's 1; beyond, the clamp only lowers a near distance: more boxes
        // kept, never fewer), so a slot costs max3 + min3 + min + compare.  s is a power of two
        // (exact), the constants' subtraction one more rounding of the origin term
        // (<= 2^-24 (|o/d| + t_min): inside the delta budget with the origin perturbation).
        constexpr float kS = kClampScale;
        const f2 sxp = {ix * kS, (-oix - tmin_lo) * kS}, syp = {iy * kS, (-oiy - tmin_lo) * kS},
                 szp = {iz * kS, (-oiz - tmin_lo) * kS};
        const f2 fxp = {ixs * kS, (-(ox_f * ixs) - tmin_lo) * kS}, fyp = {iys * kS, (-(oy_f * iys) - tmin_lo) * kS},
                 fzp = {izs * kS, (-(oz_f * izs) - tmin_lo) * kS};
#elif YK_SLAB_PAIRS_F64
        // per axis ONE register pair (1/d, -o/d) (near) and (c/d, -o c/d) (far), read by op_sel
        // (yk_slab.hpp): 12 VGPRs instead of 24
        const f2 sxp = {ix, -oix}, syp = {iy, -oiy}, szp = {iz, -oiz};
        const f2 fxp = {ixs, -(ox_f * ixs)}, fyp = {iys, -(oy_f * iys)}, fzp = {izs, -(oz_f * izs)};
#else
        const f2 ixv = {ix, ix}, iyv = {iy, iy}, izv = {iz, iz};
        const f2 noix = {-oix, -oix}, noiy = {-oiy, -oiy}, noiz = {-oiz, -oiz};
        const f2 ixc = {ixs, ixs}, iyc = {iys, iys}, izc = {izs, izs};
        const f2 noixc = {-(ox_f * ixs), -(ox_f * ixs)}, noiyc = {-(oy_f * iys), -(oy_f * iys)},
                 noizc = {-(oz_f * izs), -(oz_f * izs)};
#endif
        const double ia = ykd::rcp_bound(a);  // bounds only: relative error < 2^-44
        double ustar = INFINITY;  // proven upper bound of the minimum exact root
        float ustar_f = INFINITY;  // >= ustar * (1 + 2^-18) (YK_NEAR_CLAMP: >= s (that - tmin_lo))
#if YK_SLAB_PAIRS_F64 && YK_NEAR_CLAMP
        // a lane whose 1/d could leave float's normal range once scaled (|d| >= 1e30, never seen)
        // is marked for the exact linear scan from the start (nc = 5, as an overflow)
#if YK_CAND_PACK
        // the candidates' tuple ids as 16-bit halves (ids are < 2^16: ykgpu_set_scene's limit),
        // entry 0 in cp01's low half
        uint32_t nc = dmax < 1e30f ? 0u : 5u, cp01 = 0, cp23 = 0;
#else
        uint32_t nc = dmax < 1e30f ? 0u : 5u, c0 = 0, c1 = 0, c2 = 0, c3 = 0;
#endif
#if YK_CAND_HD
        // hb and disc of entry 0 (always the newest candidate: a compaction is followed by the
        // insertion that caused it), so its exact root needs no second discriminant
        double hb0 = 0, disc0 = 0;
#if YK_CAND_RSQ
        double rsq0 = 0;  // ... and its v_rsq_f64
#endif
#endif
#else
        uint32_t nc = 0, c0 = 0, c1 = 0, c2 = 0, c3 = 0;
#endif
        // candidate lower bounds kept as floats RN(L), compared with ustar_f >= RN(U*): by
        // monotone rounding (all bounds >= 0) L <= U* implies RN(L) <= ustar_f, so the float
        // comparison only ever keeps MORE candidates than the double comparison would
        float l0 = 0, l1 = 0, l2 = 0, l3 = 0;
        // overflow of the stack or of the candidate list is recorded as nc = 5, not as a flag of
        // its own: a bool carried round the traversal loop lives in a lane mask that every
        // divergent exit has to merge (-3.4% as a bool), an integer flag is one more loop-carried
        // register (nc = 5 instead: -0.8%)
        int32_t node = ka.bvh_root;
#if YK_NODE_BF
        // this lane's traversal stack top as an LDS byte address (entries kBlk words apart), above
        // the sentinel
        // (YK_NODE_BF 2: the variable holds the address of the entry BELOW the top, kTopOff less,
        // so the visit's read of that entry and the pushes at the top take constant DS offsets)
        constexpr uint32_t kTopOff = YK_NODE_BF == 2 ? kBlk * 4u : 0u;
        const uint32_t stk_b = (uint32_t)(uintptr_t)stk;
        uint32_t top = stk_b + kBlk * 4u - kTopOff;
        const uint32_t stk_cap = stk_b + ka.stack_cap * kBlk * 4u - kTopOff;
#define YK_STK(a) (*(__attribute__((address_space(3))) int32_t*)(uintptr_t)(a))
#else
        int32_t* top = stk;  // this lane's traversal stack top (entries kBlk words apart)
        const int32_t* const stk_cap = stk + ka.stack_cap * kBlk;
#endif
        for (;;) {
          if (node >= 0) {
#if YK_NODE_BF
           // the lane's run of interior nodes as a loop of its own tested at the bottom: its exit
           // value is the visit's own result, so the compiler keeps node / top / nc in place
#if YK_VISIT_UNSWITCH
           // (two copies of the loop, with and without the stack check: no uniform branch inside)
           auto visit_run = [&](auto chk) __attribute__((always_inline)) {
#endif
           do {
#endif
            if (kCount) ++n_node;
            YK_STAMP_NODE_ITERATION(lane);
#if YK_NODE_BF
            // the entry below the top (the sentinel when the stack holds nothing), read with the
            // planes: the pushes below write at and above the top, never here
            const int32_t popped = YK_STK(top + kTopOff - kBlk * 4u);
#endif
            // near / far distances of the 4 slots per axis, one packed FMA per pair of slots:
            // t = plane*(1/d) - o*(1/d), the binary node's arithmetic per slot
            const f4 qnx = *(const f4*)(px + node), qfx = *(const f4*)(px + node + 16);
            const f4 qny = *(const f4*)(py + node), qfy = *(const f4*)(py + node + 16);
            const f4 qnz = *(const f4*)(pz + node), qfz = *(const f4*)(pz + node + 16);
#if YK_NODE_BF
            // the scene's LDS copy starts at LDS address 0 (the kernel's only LDS is the dynamic
            // region, checked at the kernel's start), so the child codes of node n sit at n + 144
            int4 ch;
            if (kSceneInLds) {
              typedef int i4v __attribute__((ext_vector_type(4)));
              const i4v c4 = *(__attribute__((address_space(3))) const i4v*)(uintptr_t)((uint32_t)node + 144u);
              ch = make_int4(c4.x, c4.y, c4.z, c4.w);
            } else {
              ch = *(const int4*)(nodes + node + 144);
            }
#else
            const int4 ch = *(const int4*)(nodes + node + 144);
#endif
            bool hk[4];
#if YK_SLAB_PAIRS_F64 && YK_NEAR_CLAMP
            const f2 nx[2] = {slab_fma_clamp(qnx.xy, sxp), slab_fma_clamp(qnx.zw, sxp)};
            const f2 fx[2] = {slab_fma(qfx.xy, fxp), slab_fma(qfx.zw, fxp)};
            const f2 ny[2] = {slab_fma_clamp(qny.xy, syp), slab_fma_clamp(qny.zw, syp)};
            const f2 fy[2] = {slab_fma(qfy.xy, fyp), slab_fma(qfy.zw, fyp)};
            const f2 nz[2] = {slab_fma_clamp(qnz.xy, szp), slab_fma_clamp(qnz.zw, szp)};
            const f2 fz[2] = {slab_fma(qfz.xy, fzp), slab_fma(qfz.zw, fzp)};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              float tna, tfa, tnb, tfb;
              slab_cull2c(nx[h][0], ny[h][0], nz[h][0], fx[h][0], fy[h][0], fz[h][0], nx[h][1], ny[h][1], nz[h][1],
                          fx[h][1], fy[h][1], fz[h][1], ustar_f, tna, tfa, tnb, tfb);
              hk[2 * h] = tna <= tfa;
              hk[2 * h + 1] = tnb <= tfb;
            }
#elif YK_SLAB_PAIRS_F64
            const f2 nx[2] = {slab_fma(qnx.xy, sxp), slab_fma(qnx.zw, sxp)};
            const f2 fx[2] = {slab_fma(qfx.xy, fxp), slab_fma(qfx.zw, fxp)};
            const f2 ny[2] = {slab_fma(qny.xy, syp), slab_fma(qny.zw, syp)};
            const f2 fy[2] = {slab_fma(qfy.xy, fyp), slab_fma(qfy.zw, fyp)};
            const f2 nz[2] = {slab_fma(qnz.xy, szp), slab_fma(qnz.zw, szp)};
            const f2 fz[2] = {slab_fma(qfz.xy, fzp), slab_fma(qfz.zw, fzp)};
#if YK_CULL_BLOCK
            // two slots per asm block (yk_slab.hpp slab_cull2): the same instructions, fewer edges
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              float tna, tfa, tnb, tfb;
              slab_cull2(nx[h][0], ny[h][0], nz[h][0], fx[h][0], fy[h][0], fz[h][0], nx[h][1], ny[h][1], nz[h][1],
                         fx[h][1], fy[h][1], fz[h][1], tmin_lo, ustar_f, tna, tfa, tnb, tfb);
              hk[2 * h] = tna <= tfa;
              hk[2 * h + 1] = tnb <= tfb;
            }
#else
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const float tn = slab_max(slab_max3(nx[k >> 1][k & 1], ny[k >> 1][k & 1], nz[k >> 1][k & 1]), tmin_lo);
              const float tf = slab_min(slab_min3(fx[k >> 1][k & 1], fy[k >> 1][k & 1], fz[k >> 1][k & 1]), ustar_f);
              hk[k] = tn <= tf;
            }
#endif
#else
            const f2 nx[2] = {__builtin_elementwise_fma(qnx.xy, ixv, noix), __builtin_elementwise_fma(qnx.zw, ixv, noix)};
            const f2 fx[2] = {__builtin_elementwise_fma(qfx.xy, ixc, noixc), __builtin_elementwise_fma(qfx.zw, ixc, noixc)};
            const f2 ny[2] = {__builtin_elementwise_fma(qny.xy, iyv, noiy), __builtin_elementwise_fma(qny.zw, iyv, noiy)};
            const f2 fy[2] = {__builtin_elementwise_fma(qfy.xy, iyc, noiyc), __builtin_elementwise_fma(qfy.zw, iyc, noiyc)};
            const f2 nz[2] = {__builtin_elementwise_fma(qnz.xy, izv, noiz), __builtin_elementwise_fma(qnz.zw, izv, noiz)};
            const f2 fz[2] = {__builtin_elementwise_fma(qfz.xy, izc, noizc), __builtin_elementwise_fma(qfz.zw, izc, noizc)};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const float tn = fmaxf(fmaxf(fmaxf(nx[k >> 1][k & 1], ny[k >> 1][k & 1]), nz[k >> 1][k & 1]), tmin_lo);
              const float tf = fminf(fminf(fminf(fx[k >> 1][k & 1], fy[k >> 1][k & 1]), fz[k >> 1][k & 1]), ustar_f);
              hk[k] = tn <= tf;
            }
#endif
            // keep the child-code read in this block, issued with the plane reads (the compiler
            // would otherwise sink it into the branch below and wait for it there)
            asm volatile("" ::"v"(ch.x), "v"(ch.y), "v"(ch.z), "v"(ch.w));
#if YK_NODE_BF
            {
              // the last slot entered is visited next, the others entered are pushed in slot
              // order; none entered: the popped entry is next and the top moves down one
              const bool any = hk[0] || hk[1] || hk[2] || hk[3];
              node = hk[3] ? ch.w : (hk[2] ? ch.z : (hk[1] ? ch.y : (hk[0] ? ch.x : popped)));
              YK_STK(top + kTopOff) = ch.x;
              top += (hk[0] && (hk[1] || hk[2] || hk[3])) ? kBlk * 4u : 0u;
              YK_STK(top + kTopOff) = ch.y;
              top += (hk[1] && (hk[2] || hk[3])) ? kBlk * 4u : 0u;
              YK_STK(top + kTopOff) = ch.z;
              top += (hk[2] && hk[3]) ? kBlk * 4u : (any ? 0u : 0u - kBlk * 4u);
              // stack full: the top stays at the capacity and nc = 5 sends the lane to the scan
              // (only where the plan could not give the stack its proven depth: ka.stack_check)
#if YK_VISIT_UNSWITCH
              if (decltype(chk)::value) {
#else
              if (ka.stack_check) {
#endif
                asm volatile("");  // (a scalar branch: no selects on the uniform flag)
                // signed: with YK_NODE_BF 2 the pop of the sentinel leaves `top` one entry below the
                // stack's base, below LDS address 0 for the low lanes of a scene with a small LDS
                // copy (unsigned, that wrapped past the capacity and the lane never left the loop)
                nc = (int32_t)top > (int32_t)stk_cap ? 5u : nc;
                top = (int32_t)top > (int32_t)stk_cap ? stk_cap : top;
              }
            }
           } while (node >= 0);
#if YK_VISIT_UNSWITCH
           };
           if (ka.stack_check) visit_run(std::true_type{}); else visit_run(std::false_type{});
#endif
#else
            if (hk[0] || hk[1] || hk[2] || hk[3]) {
              // the last slot entered is visited next and the others entered are pushed, in slot
              // order: no distance sort (visit order only affects how fast U* shrinks, never the
              // result; modelled by tools/bvhsim, it costs ~1% more leaf tests and no node
              // visits).  Each write lands at the current top, which moves only for a push.
              node = hk[3] ? ch.w : (hk[2] ? ch.z : (hk[1] ? ch.y : ch.x));
              *top = ch.x;
              top += (hk[0] && (hk[1] || hk[2] || hk[3])) ? kBlk : 0;
              *top = ch.y;
              top += (hk[1] && (hk[2] || hk[3])) ? kBlk : 0;
              *top = ch.z;
              top += (hk[2] && hk[3]) ? kBlk : 0;
              // stack full: the top stays at the capacity (the pushes above it are lost and the
              // rest of this traversal is void) and nc = 5 marks the lane for the exact linear scan
              if (top > stk_cap) {
                top = stk + ka.stack_cap * kBlk;
                nc = 5;
              }
              continue;
            }
            // no slot entered: pop here, inside the visit branch, so the lane goes on with the
            // popped node in the next trip instead of waiting for every other lane of the wave to
            // stop descending (512 spp: 180.8 -> 178.4 ms); an empty stack ends the traversal as
            // the empty leaf (~0: no spheres)
            if (top == stk) {
              node = ykbvh::kEmptyLeaf;
            } else {
              top -= kBlk;
              node = *top;
            }
            continue;
#endif
#if YK_NODE_BF
          }
          {
#else
          } else {
#endif
            YK_STAMP(2);  // interior nodes since the last stamp
            const uint32_t v = ~(uint32_t)node, first = v >> 4, cnt = v & 15u;
            // the FP64 tree has one sphere per leaf (max_leaf = 1: the builder's median fallback
            // never leaves more), so a leaf is tested without a loop (512 spp: -0.9%); the empty
            // leaf ~0 (cnt 0) tests nothing.  (`continue` inside the do-while(0) leaves the test.)
            static_assert(kLeafCapF64 == 1, "the FP64 leaf test handles one sphere");
            if (cnt != 0) do {
              const uint32_t k = 0;
              const SphereGeo sg = leaf_geo[first + k];
              // the tuple index read with the geometry: its latency then hides under the
              // discriminant instead of following the bounds on the insert path
              const uint32_t id = leaf_ids[first + k];
              asm volatile("" ::"v"(id));
              ++n_test;
              // the reference's discriminant, bit for bit (sphere.hpp:29-34)
              const v3 oc = {o.x - sg.cx, o.y - sg.cy, o.z - sg.cz};
              const double hb = ykd::dot(oc, d);
              const double c = ykd::len2(oc) - sg.rr;
              const double disc = hb * hb - a * c;
              if (disc < 0) continue;
              if (kCount) ++n_dpos;
              YK_STAMP_DISC_POS();
              // bounds of the exact root: |approx - exact| <= m (256x the error bound, §4)
#if YK_CAND_HD && YK_CAND_RSQ
              const double rq = __builtin_amdgcn_rsq(disc);
              const double sq = ykd::sqrt_bound_r(disc, rq);
#else
              const double sq = ykd::sqrt_bound(disc);
#endif
              const double r1 = (-hb - sq) * ia, r2 = (-hb + sq) * ia;
              const double m = (fabs(hb) + sq) * ia * 0x1p-34 + 0x1p-1000;
              if (r2 + m < ka.t_min) continue;  // both roots certainly behind t_min
              const double lb = fmax(ka.t_min, r1 - m);
              const double ub = (r1 - m >= ka.t_min) ? r1 + m : ((r2 - m >= ka.t_min) ? r2 + m : INFINITY);
              if (!(lb <= ustar)) continue;
              if (ub < ustar) {
                ustar = ub;
#if YK_SLAB_PAIRS_F64 && YK_NEAR_CLAMP
                // s (RN(ub)(1 + 2^-18) - tmin_lo), rounded up by the factor 1 + 2^-22: >= s (the
                // unshifted bound - tmin_lo), positive (ub >= t_min > tmin_lo)
                ustar_f = ((float)ub * (1.0f + 0x1p-18f) - tmin_lo) * ((1.0f + 0x1p-22f) * kClampScale);
#else
                ustar_f = (float)ub * (1.0f + 0x1p-18f);
#endif
              }
              if (nc == 4) {  // compact: drop entries the new bound has excluded
                uint32_t m2 = 0;
#if YK_CAND_PACK
                uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0;
                const uint32_t d0 = cp01 & 0xffffu, d1 = cp01 >> 16, d2 = cp23 & 0xffffu, d3 = cp23 >> 16;
#else
                uint32_t d0 = c0, d1 = c1, d2 = c2, d3 = c3;
#endif
                float e0 = l0, e1 = l1, e2 = l2, e3 = l3;
                if (e0 <= ustar_f) { YK_CAND_SET(m2, d0, e0); ++m2; }
                if (e1 <= ustar_f) { YK_CAND_SET(m2, d1, e1); ++m2; }
                if (e2 <= ustar_f) { YK_CAND_SET(m2, d2, e2); ++m2; }
                if (e3 <= ustar_f) { YK_CAND_SET(m2, d3, e3); ++m2; }
                nc = m2;
#if YK_CAND_PACK
                cp01 = c0 | (c1 << 16);
                cp23 = c2 | (c3 << 16);
#endif
              }
              if (nc < 4) {
                // shifted in at entry 0 — straight-line moves instead of a branch per list
                // position (evaluation order never matters: min root, later index on ties).
                // RN(lb), not rounded down: t_min >= 0 (checked by the host) makes every lb and
                // U* >= 0, and lb <= U* implies RN(lb) <= RN(U*) <= ustar_f (monotone rounding),
                // so the list still keeps every sphere that can be the minimum
#if YK_CAND_PACK
                cp23 = __builtin_amdgcn_alignbit(cp23, cp01, 16u);  // (cp23 << 16) | (cp01 >> 16)
                cp01 = (cp01 << 16) | id;
                l3 = l2, l2 = l1, l1 = l0;
#else
                c3 = c2, l3 = l2, c2 = c1, l2 = l1, c1 = c0, l1 = l0;
#endif
#if YK_CAND_HD
                hb0 = hb, disc0 = disc;
#if YK_CAND_RSQ
                rsq0 = rq;
#endif
#endif
#if YK_SLAB_PAIRS_F64 && YK_NEAR_CLAMP
                // the same monotone map as ustar_f's: s RN(RN(lb) - tmin_lo) (one FMA, s a power of
                // two), so lb <= U* still implies l0 <= ustar_f
#if YK_CAND_PACK
                l0 = __builtin_fmaf((float)lb, kClampScale, -tmin_lo * kClampScale);
#else
                c0 = id, l0 = __builtin_fmaf((float)lb, kClampScale, -tmin_lo * kClampScale);
#endif
#else
                c0 = id, l0 = (float)lb;
#endif
                ++nc;
              } else {
                nc = 5;  // the list is full: overflow (the exact linear scan decides)
              }
            } while (0);
            YK_STAMP(6);  // this leaf
          }
#if YK_NODE_BF
          if (top + kTopOff <= stk_b + kBlk * 4u) break;  // only the sentinel left, or the sentinel just visited
          top -= kBlk * 4u;
          node = YK_STK(top + kTopOff);
#undef YK_STK
#else
          if (top == stk) break;
          top -= kBlk;
          node = *top;
#endif
        }
        YK_STAMP(2);
        if (nc > 4) {
          linear = true;
        } else {
          // exact evaluation of the survivors; the roots' divisor a is the same for every
          // candidate of a ray, so its refined reciprocal is computed once
          const bool a_ok = ykd::div_range(a);
#if YK_RA_FROM_IA
          // rcp_refined(a)'s first Newton step is rcp_bound(a) = ia, bit for bit (the same rcp and
          // fmas): the second step alone (YK_RA_FROM_IA)
          const double ra = (nc > 0 && a_ok) ? __builtin_fma(ia, __builtin_fma(-a, ia, 1.0), ia) : 0.0;
#else
          const double ra = (nc > 0 && a_ok) ? ykd::rcp_refined(a) : 0.0;
#endif
#if YK_CAND_HD
#if YK_CAND_PACK
          const uint32_t c0 = cp01 & 0xffffu, c1 = cp01 >> 16, c2 = cp23 & 0xffffu, c3 = cp23 >> 16;
#endif
#if YK_CAND_RSQ
          if (nc > 0 && l0 <= ustar_f) exact_root(c0, hb0, disc0, a, ra, a_ok, ka.t_min, hit, &rsq0);
#else
          if (nc > 0 && l0 <= ustar_f) exact_root(c0, hb0, disc0, a, ra, a_ok, ka.t_min, hit);
#endif
#else
          if (nc > 0 && l0 <= ustar_f) exact_candidate(geo, c0, o, d, a, ra, a_ok, ka.t_min, hit);
#endif
          if (nc > 1 && l1 <= ustar_f) exact_candidate(geo, c1, o, d, a, ra, a_ok, ka.t_min, hit);
          if (nc > 2 && l2 <= ustar_f) exact_candidate(geo, c2, o, d, a, ra, a_ok, ka.t_min, hit);
          if (nc > 3 && l3 <= ustar_f) exact_candidate(geo, c3, o, d, a, ra, a_ok, ka.t_min, hit);
        }
      }
      if (linear) {
        hit = scan_linear(ka.geo, ka.nspheres, o, d, ka.t_min);
        n_test += hit.tests;
        ++n_lin;
      }
      n_sqrt += hit.sqrts;
      n_ncall += hit.ncalls;
      n_nit += hit.nits;
    }
    YK_STAMP(3);

    // (b) shade, material-uniform: every operation more than one material needs runs ONCE for all
    //     the lanes that need it, instead of once per material branch (a wave holds every kind
    //     almost every trip, so per-branch copies run one after the other):
    //   * one block of canonicals: lambertian's vec3::random (3), the fuzzed metal's length factor
    //     and vector (4), the dielectric's reflect-or-refract uniform (1, drawn speculatively:
    //     given back when total internal reflection means the reference never draws it);
    //   * one vector normalisation — the sky's normalized(dir) (raytracer.hpp:35), lambertian's
    //     random_unit_vector (material.hpp:33-36), metal's / dielectric's normalized(dir);
    //   * one more Newton square root: the fuzzed metal's |vector| or the dielectric's sin(theta).
    //   Each lane's own operations and their order are the reference's.
    bool ended = in_path && !alive;
    double L_r = 0, L_g = 0, L_b = 0;
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
        // hit record (sphere.hpp:41-45, hittable.hpp:23-27)
        p = ykd::add(o, ykd::mul(d, T));
        const v3 outward = ykd::divs_fast_r(ykd::sub(p, v3{sg.cx, sg.cy, sg.cz}), m.radius, m.inv_r);
        front = ykd::dot(d, outward) < 0;
        nrm = front ? outward : ykd::neg(outward);
      }
      const bool lamb = hid >= 0 && m.kind == YK_MATERIAL_LAMBERTIAN;
      const bool fuzzy = hid >= 0 && m.kind == YK_MATERIAL_METAL && m.fuzz > 0;
      const bool diel = hid >= 0 && m.kind == YK_MATERIAL_DIELECTRIC;
      const bool spec = diel && ykd::rng_can_speculate(g);
      const Gen saved = g;  // the dielectric's engine before its speculative draw
      const uint32_t ncan = lamb ? 3u : (fuzzy ? 4u : (spec ? 1u : 0u));
      double c0 = 0, c1 = 0, c2 = 0, c3 = 0;
      if (__ballot(ncan > 0 && !ykd::rng_lazy_ok(g, 2 * ncan)) == 0) {
        // (almost always) no lane of the wave reaches the scratch engine's words: no checks
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
      // lambertian: vec3::random(gen, -1, 1), x then y then z (vec3.hpp:134-142); fuzzed metal:
      // random(-1,1).normalize() * uniform(0.01,0.99) with the factor drawn first — g++, the
      // reference's compiler, evaluates that product's operands right to left (pinned by the
      // reference-harness goldens, tests/golden/gen_golden.py)
      const v3 rv = lamb ? v3{ykd::uniform_of(c0, -1, 1), ykd::uniform_of(c1, -1, 1), ykd::uniform_of(c2, -1, 1)}
                         : v3{ykd::uniform_of(c1, -1, 1), ykd::uniform_of(c2, -1, 1), ykd::uniform_of(c3, -1, 1)};
      const v3 vn = lamb ? rv : d;
      const double len = ykd::nsqrt_c(ykd::len2(vn), n_ncall, n_nit);  // vec3::length(), vec3.hpp:127
      // vn / len is what every branch below divides (sky: d.y / len; lambertian: the random
      // vector; metal, dielectric: d), so it is computed once here, not once per branch
      const v3 un = ykd::divs_fast(vn, len);
      double ct = 0;  // dielectric: cos(theta) = min(dot(-unit, n), 1)
      if (diel) {
        ct = ykd::dot(ykd::neg(un), nrm);
        if (!(ct < 1.0)) ct = 1.0;
      }
      double sq2 = 0;  // fuzzed metal: |random vector|; dielectric: sin(theta)
      if (fuzzy || diel) sq2 = ykd::nsqrt_c(fuzzy ? ykd::len2(rv) : 1.0 - ct * ct, n_ncall, n_nit);
      if (hid < 0) {
        // sky (raytracer.hpp:35-36): t = (normalized(dir).y + 1)/2, lerp white → (.5,.7,1)
        const double t = (un.y + 1.0) / 2;
        L_r = (1.0 - t) * 1.0 + t * 0.5;
        L_g = (1.0 - t) * 1.0 + t * 0.7;
        L_b = (1.0 - t) * 1.0 + t * 1.0;
        ended = true;
      } else {
        bool scattered = true, push = true;
        v3 nd;
        if (m.kind == YK_MATERIAL_LAMBERTIAN) {  // material.hpp:50-59
          if (kCount) ++n_lamb;
          nd = ykd::add(nrm, un);
          if (ykd::near_zero(nd)) nd = nrm;
        } else if (m.kind == YK_MATERIAL_METAL) {  // material.hpp:67-75 (+ fuzz extension)
          if (kCount) ++n_metal;
          nd = ykd::reflect(un, nrm);
          if (fuzzy) {  // + fuzz * random_in_unit_sphere (material.hpp:27-30)
            if (kCount) ++n_fuzz;
            const double k = ykd::uniform_of(c0, 0.01, 0.99);
            const v3 ru = ykd::divs_fast(rv, sq2);
            nd = ykd::add(nd, ykd::mul(ykd::mul(ru, k), m.fuzz));
          }
          scattered = ykd::dot(nd, nrm) > 0;
        } else {  // dielectric extension (attenuation (1,1,1): multiplying by 1.0 is exact)
          if (kCount) ++n_diel;
          push = false;
#if YK_DIEL_PRE
          // 1/ior and Schlick's r0 of both sides precomputed on the host with the same IEEE
          // operations (ykgpu_set_scene: the dielectric's unused fuzz / albedo fields)
          const double ratio = front ? m.fuzz : m.ior;
          const double r0 = front ? m.ar : m.ag;
#else
          const double ratio = front ? (1.0 / m.ior) : m.ior;
#endif
          const v3 unit = un;
          const double sn = sq2;
          const bool cannot = ratio * sn > 1.0;
          double u = 0;
          if (cannot) {
            if (spec) g = saved;  // `cannot || ...` never draws: give the word pair back
          } else {
            u = spec ? ykd::uniform_of(c0, 0, 1) : ykd::uniform(g, 0, 1);
          }
#if YK_DIEL_PRE
          if (cannot || ykd::reflectance_r0(ct, r0) > u) {
#else
          if (cannot || ykd::reflectance(ct, ratio) > u) {
#endif
            nd = ykd::reflect(unit, nrm);
          } else {
            const v3 perp = ykd::mul(ykd::add(unit, ykd::mul(nrm, ct)), ratio);
            const double pl = 1.0 - ykd::len2(perp);
            nd = ykd::add(perp, ykd::mul(nrm, -ykd::nsqrt_c(pl < 0 ? -pl : pl, n_ncall, n_nit)));
          }
        }
        if (!scattered) {
          ended = true;  // absorbed: black (raytracer.hpp:30)
        } else {
          if (push) {
            if (nstk >= kStackRegs) id_spill[nstk - kStackRegs] = (uint16_t)(st3 >> 16);
            st3 = (st3 << 16) | (st2 >> 16);
            st2 = (st2 << 16) | (st1 >> 16);
            st1 = (st1 << 16) | (st0 >> 16);
            st0 = (st0 << 16) | (uint32_t)hid;
            ++nstk;
          }
          o = p;
          d = nd;
          --depth;
        }
      }
    }
    YK_STAMP(4);

    if (ended) {
      // unwind: attenuation_k * (...) from the deepest scatter outwards (raytracer.hpp:31)
      auto pop = [&]() {
        const uint32_t id = st0 & 0xffffu;
        st0 = (st0 >> 16) | (st1 << 16);
        st1 = (st1 >> 16) | (st2 << 16);
        st2 = (st2 >> 16) | (st3 << 16);
        st3 = (st3 >> 16) | (nstk > kStackRegs ? ((uint32_t)id_spill[nstk - kStackRegs - 1] << 16) : 0u);
        --nstk;
        return id;
      };
#if YK_UNWIND_FAST
      if (__ballot(nstk > kStackRegs) == 0) {
        // no ending lane of the wave holds spilled ids: the register window alone, two ids per
        // round (the window moves by a whole register)
        while (nstk > 0) {
          const SphereMat m = mat[st0 & 0xffffu];
          L_r = m.ar * L_r;
          L_g = m.ag * L_g;
          L_b = m.ab * L_b;
          if (nstk > 1) {
            const SphereMat m2 = mat[st0 >> 16];
            L_r = m2.ar * L_r;
            L_g = m2.ag * L_g;
            L_b = m2.ab * L_b;
          }
          st0 = st1, st1 = st2, st2 = st3;
          nstk = nstk > 1 ? nstk - 2 : 0;
        }
      } else
#endif
      while (nstk > 0) {
        const SphereMat m = mat[pop()];
        L_r = m.ar * L_r;
        L_g = m.ag * L_g;
        L_b = m.ab * L_b;
      }
      if (ykd::mt_used_fallback(g)) ++n_fb;
      if (kCount) n_words += ykd::rng_words(g), n_twist += ykd::rng_twists(g);
      // the sample's colour; yk_reduce_samples adds them in sample order
      colour_store(ka.col, slot, L_r, L_g, L_b);
      in_path = false;
    }
    YK_STAMP(5);
  }

  YK_CLOCK_END(ka);
  YK_WAVE_STAMP(ka, 1);
  YK_STAMPS_END(ka.counters, lane);
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
    atomicAdd(&ka.counters[29], (unsigned long long)n_words);
    atomicAdd(&ka.counters[30], (unsigned long long)n_swords);
    atomicAdd(&ka.counters[31], (unsigned long long)n_twist);
  }
  if (n_fb) atomicAdd(&ka.counters[3], (unsigned long long)n_fb);
#if YK_WG_HOLD
  // (A/B) the workgroup's waves leave together: a wave without work keeps its registers until the
  // last one is done, so the CU frees whole and the next launch's workgroup is not starved by the
  // warm-up's small workgroups taking the registers piecemeal
  if constexpr (kMode == 0) __syncthreads();
#endif
}


// The kernels.  Production instances at <= YK_RENDER_VGPRS (gfx950's amdgpu_num_vgpr counts the
// unified file, so the attribute takes half).
template <bool kSceneInLds, int kMode>
__global__ __launch_bounds__(mode_block<kMode>())
#if YK_WAVES_PER_EU
__attribute__((amdgpu_waves_per_eu(YK_WAVES_PER_EU, YK_WAVES_PER_EU)))
#else
__attribute__((amdgpu_waves_per_eu(4, 8)))
#endif
#ifdef YK_SINGLE_VGPRS
__attribute__((amdgpu_num_vgpr(YK_SINGLE_VGPRS / 2)))  // (A/B)
#else
__attribute__((amdgpu_num_vgpr(YK_RENDER_VGPRS / 2)))
#endif
void yk_render_persistent(KernelArgs ka) {
  render_body<kSceneInLds, kMode>(ka);
}
// the counting instances (kMode bit 0: diagnostic builds of the same body, YK_FLAG_COUNT_WORK)
// under a name of their own, their registers uncapped
template <bool kSceneInLds, int kMode>
__global__ __launch_bounds__(mode_block<kMode>()) __attribute__((amdgpu_waves_per_eu(1, 8)))
void yk_render_counting(KernelArgs ka) {
  render_body<kSceneInLds, kMode>(ka);
}

// The FP64 instance for (scene in LDS, kMode)
RenderKernel fp64_kernel(bool lds, int mode) {
  static const RenderKernel k[16] = {
      yk_render_persistent<false, 0>, yk_render_counting<false, 1>,  yk_render_persistent<false, 2>,
      yk_render_counting<false, 3>,   yk_render_persistent<false, 4>, yk_render_counting<false, 5>,
      yk_render_persistent<false, 6>, yk_render_counting<false, 7>,  yk_render_persistent<true, 0>,
      yk_render_counting<true, 1>,    yk_render_persistent<true, 2>,  yk_render_counting<true, 3>,
      yk_render_persistent<true, 4>,  yk_render_counting<true, 5>,    yk_render_persistent<true, 6>,
      yk_render_counting<true, 7>};
  return k[(lds ? 8 : 0) + (mode & 7)];
}

#endif  // YK_SPLIT != 2

#if YK_SPLIT != 1

// ---- render<float> (YK_PRECISION_FP32) ---------------------------------------------------
// The same persistent, sample-parallel structure as yk_render_persistent (refill, slots, start
// records from yk_mt_warmup, attenuation-id stack, SoA colours reduced by yk_reduce_samples),
// with the path in float (yk_device_f32.hpp).  Closest hit: the FP32 tree culls — its boxes and
// a per-ray cone carry the float sphere test's proven error — the spheres of an
// entered leaf get the reference's float discriminant and bounds of their float root, and the
// survivors' exact float roots are evaluated after the traversal: the minimum root wins, an exact
// tie goes to the later tuple index.  Rays outside the tree's proven range take the ordered scan
// (hittable_list.hpp:32-58).
template <class G>
__device__ __forceinline__ float f_uniform01(G& g) { return ykf::uniform(g, 0.0f, 1.0f); }

// sphere::hit_impl<float> (sphere.hpp:25-48) bit for bit, without t_max.  Returns 2 with the root
// in r (root1 if >= tmin, else root2: the reference accepts it iff r <= t_max, because root2 >=
// root1 under monotonic rounding), 1 when both roots lie below tmin, 0 when disc < 0.
// n / a for a root, a's refined reciprocal ra shared by the ray's candidates (ykf::div_by); a wave
// with any lane out of range takes the full division
__device__ __forceinline__ float f32_root_div(float n, float a, float ra, bool a_ok) {
  float q = ykf::div_by(n, a, ra);
  if (__builtin_expect(__ballot(!(a_ok && ykf::num_range(n))) != 0, 0)) q = n / a;
  return q;
}
__device__ __forceinline__ int f32_root(float4 sg, ykf::v3 o, ykf::v3 d, float a, float ra, bool a_ok, float tmin,
                                        float& r, uint32_t& nit) {
  const ykf::v3 oc = {o.x - sg.x, o.y - sg.y, o.z - sg.z};
  const float hb = ykf::dot(oc, d);
  const float c = ykf::len2(oc) - sg.w;
  const float disc = hb * hb - a * c;
  if (disc < 0) return 0;
  const float sq = ykf::nsqrt(disc, nit);
  r = f32_root_div(-hb - sq, a, ra, a_ok);
  if (r < tmin) {
    r = f32_root_div(-hb + sq, a, ra, a_ok);
    if (r < tmin) return 1;
  }
  return 2;
}

// the cone keeps a far bound on an axis with |d| >= kF32FarAt s, and gives the slow-axis bound
// to one with |d| < kF32SlowAt s (d - s sign d stays clear of 0 in both)
constexpr float kF32FarAt = 1.0f + 0x1p-10f, kF32SlowAt = 1.0f - 0x1p-10f;

// Bounds of the root f32_root returns, from the exact float discriminant: the
// approximation r = (-hb ∓ v_sqrt_f32(disc)) · v_rcp_f32(a) differs from the exact root by at most
// (|hb| + √disc)/a · 9u (one-step sqrt within 1.5u, v_sqrt/v_rcp within an ulp, three roundings;
// u = 2^-24); m takes 256u, plus an absolute term for underflowing products.  A disc outside the
// one-step square root's range [2^-100, 2^100] gets no bound (m = inf: always a candidate).
// Returns false when both roots certainly lie below tmin; else lb <= the accepted root <= ub
// (ub = inf when neither root is certainly >= tmin).  NaN anywhere keeps the sphere (every
// comparison that would drop it is false).
__device__ __forceinline__ bool f32_root_bounds(float hb, float disc, float ia, float tmin, float& lb, float& ub) {
  const float sq = __builtin_amdgcn_sqrtf(disc);
  const float r1 = (-hb - sq) * ia, r2 = (-hb + sq) * ia;
  float m = (fabsf(hb) + sq) * ia * 0x1p-16f + 0x1p-120f;
  if (!(disc >= 0x1p-100f && disc <= 0x1p100f)) m = INFINITY;
  if (r2 + m < tmin) return false;
  lb = fmaxf(tmin, r1 - m);
  ub = (r1 - m >= tmin) ? r1 + m : ((r2 - m >= tmin) ? r2 + m : INFINITY);
  return true;
}

// One axis of the ray's cone: near planes are crossed at (plane - o) * in, far
// planes at (plane - o) * jf, with in = 1/(d + s sign d) and jf = (1 + 2^-17)/(d - s sign d); an
// axis with |d| < kF32FarAt s keeps no far bound (jf = 0, constant +inf).  Slab FMA operands:
// plane * in + nc.  Culling arithmetic only: v_rcp_f32's ulp is inside the relative margins (d - s
// sign d is exact for |d| <= 2s, Sterbenz).
__device__ __forceinline__ void cone_axis(float dk, float ok, float s, f2& in2, f2& nc2, f2& jf2, f2& fc2) {
  const float sg = dk < 0.0f ? -s : s;
  const float in = __builtin_amdgcn_rcpf(dk + sg);
  const bool far = fabsf(dk) >= kF32FarAt * s;
  const float jf = far ? __builtin_amdgcn_rcpf(dk - sg) * (1.0f + 0x1p-17f) : 0.0f;
  const float nc = -(ok * in), fc = far ? -(ok * jf) : INFINITY;
#if YK_SLAB_PAIRS_F32
  // the pairs (in, nc) and (jf, fc), read by op_sel (yk_slab.hpp); nc2 / fc2 unused
  in2 = f2{in, nc};
  jf2 = f2{jf, fc};
  nc2 = fc2 = f2{0.0f, 0.0f};
#else
  in2 = f2{in, in};
  nc2 = f2{nc, nc};
  jf2 = f2{jf, jf};
  fc2 = f2{fc, fc};
#endif
}

// kSceneInLds: the FP32 tree, its float4 leaf geometry and its leaf ids copied into LDS per
// workgroup, as in the FP64 kernel.  kMode bit 0: the work counters; bit 2: the yk::xor128
// engine (as for the FP64 kernel)
template <bool kSceneInLds, int kMode>
__global__ __launch_bounds__(mode_block<kMode>())
void yk_render_f32(KernelArgs ka) {
  constexpr int kBlk = mode_block<kMode>();
  constexpr bool kCount = (kMode & 1) != 0;
  using Gen = typename std::conditional<(kMode & 4) != 0, ykd::X128Lane, ykd::MtLane>::type;
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const char* __restrict__ nodes = (const char*)ka.nodes;
  const float4* __restrict__ leaf_geo = (const float4*)ka.leaf_geo;
  const uint32_t* __restrict__ leaf_ids = ka.leaf_ids;
  const float4* __restrict__ geo_f = ka.geo_f;  // tuple order: hit records
  const SphereMat* __restrict__ mat = ka.mat;   // shading, attenuation unwind
  if (kSceneInLds) {
    // as in the FP64 kernel: the BVH, its leaf geometry and ids, and the tuple-order tables
    const uint4* src[5] = {(const uint4*)ka.nodes, (const uint4*)ka.leaf_geo, (const uint4*)ka.leaf_ids,
                           (const uint4*)ka.geo_f, (const uint4*)ka.mat};
    const uint32_t off[5] = {0u, ka.lds_geo_off, ka.lds_ids_off, ka.lds_tgeo_off, ka.lds_mat_off};
    const uint32_t n16[5] = {(ka.n_nodes * (uint32_t)sizeof(DevNode) + 15u) / 16u, ka.nspheres,
                             (ka.nspheres + 3u) / 4u, ka.nspheres, ka.nspheres * 4u};
#pragma unroll
    for (int k = 0; k < 5; ++k) {
      uint4* dst = (uint4*)(smem + off[k]);
      for (uint32_t i = threadIdx.x; i < n16[k]; i += kBlk) dst[i] = src[k][i];
    }
    __syncthreads();
    nodes = smem;
    leaf_geo = (const float4*)(smem + ka.lds_geo_off);
    leaf_ids = (const uint32_t*)(smem + ka.lds_ids_off);
    geo_f = (const float4*)(smem + ka.lds_tgeo_off);
    mat = (const SphereMat*)(smem + ka.lds_mat_off);
  }
  int32_t* const stk = (int32_t*)(smem + ka.lds_stack_off) + threadIdx.x;  // [sp * kBlk]
#if YK_RENDER_PRIO
  __builtin_amdgcn_s_setprio(YK_RENDER_PRIO);  // over the co-resident warm-up waves, as in FP64
#endif
  YK_CLOCK_BEGIN(ka);
  Gen g;
  rng_init(g, ka, gid);
  uint16_t* const id_spill = ka.id_scratch + (size_t)gid * ka.id_stride;
  uint32_t n_seg = 0, n_test = 0, n_sqrt = 0, n_fb = 0, n_nit = 0, n_ncall = 0, n_node = 0, n_lin = 0;
  uint32_t n_words = 0, n_swords = 0, n_twist = 0;  // as in yk_render_persistent
  YK_STAMPS_BEGIN(ka.counters, lane);
  const float tmin = (float)ka.t_min;  // world.hit(r, 0.001, ...) converts to T (hittable.hpp:32)
  uint32_t slot = 0, depth = 0, nstk = 0;
  uint32_t st0 = 0, st1 = 0, st2 = 0, st3 = 0;
  ykf::v3 o = {0, 0, 0}, d = {0, 0, 0};
  bool in_path = false;
  uint32_t res_base = 0, res_left = 0;

  for (;;) {
    if (claim_slots(ka, in_path, lane, slot, res_base, res_left)) {
      YK_STAMPS_EXHAUSTED(ka.counters);
      break;
    }
    YK_STAMP(0);

    // ---- start: seed, jitter, camera<float>::get_ray (source.cpp:154-165, camera.hpp:29-32)
    bool start = !in_path;
    uint32_t qpix = 0;
    // mt19937: the start (draws and camera<float> ray) comes precomputed (yk_mt_warmup<lens,
    // true>: StartRecF), which alone says whether the slot is empty, as in the FP64 kernel
    constexpr bool kRec = std::is_same<Gen, ykd::MtLane>::value;
    uint4 rq0 = {0, 0, 0, 0}, rq1 = {0, 0, 0, 0}, rq2 = {0, 0, 0, 0};
    if (start) {
      if constexpr (kRec) {
        const uint4* rp = (const uint4*)ka.start + 3u * slot;
        rq0 = rp[0];
        rq1 = rp[1];
        rq2 = rp[2];
        asm volatile("" ::"v"(rq0.x), "v"(rq0.y), "v"(rq0.z), "v"(rq0.w), "v"(rq1.x), "v"(rq1.y),
                     "v"(rq2.x), "v"(rq2.y), "v"(rq2.z), "v"(rq2.w));
        start = rq2.w != kPadSlot;
      } else {
        const uint32_t sl = fdiv(slot, ka.nps_m, ka.nps_sh);
        qpix = ka.order[slot - sl * ka.npix_slots];
        start = qpix != kNoPixel;
      }
    }
    if (start) {
      bool pre = false;
      if constexpr (kRec) {
        StartRecF r;
        __builtin_memcpy((char*)&r, &rq0, 16);
        __builtin_memcpy((char*)&r + 16, &rq1, 16);
        __builtin_memcpy((char*)&r + 32, &rq2, 16);
        pre = r.j != kNoStart;
        if (pre) {
          if (kCount) n_swords += r.j;
          g.a0 = r.a0;
          g.a1 = r.a1;
          g.b = r.b;
          g.j = r.j;
          o = ykf::v3{r.ox, r.oy, r.oz};
          d = ykf::v3{r.dx, r.dy, r.dz};
        }
      }
      if (!pre) {
        const uint32_t sl = fdiv(slot, ka.nps_m, ka.nps_sh);
        if constexpr (kRec) qpix = ka.order[slot - sl * ka.npix_slots];
        const uint32_t s = ka.s0 + sl;
        const uint32_t tr = fdiv(qpix, ka.w_m, ka.w_sh);
        const uint32_t x = tile_col_x(ka.col_begin, ka.col_stride, ka.col_band, qpix - tr * ka.Wt);
        const uint32_t y = tile_row_y(ka.row_begin, ka.row_stride, ka.band_log2, tr);
        const uint32_t seed = ykd::sample_seed(ka.seed_mode, ka.seed_key, ka.seed0, y, x, ka.W, ka.spp, s);
        const bool lens = ka.cam.lens_radius > 0;  // (decided in double, as for the warm-up)
        rng_start_full(g, seed);
        const float uc = f_uniform01(g);
        const float vc = f_uniform01(g);
        float px = 0, py = 0;
        if (lens) {  // thin-lens extension: random_in_unit_disk by rejection, x then y
          do {
            px = ykf::uniform(g, -1.0f, 1.0f);
            py = ykf::uniform(g, -1.0f, 1.0f);
          } while (!(px * px + py * py < 1.0f));
        }
        camera_ray_f32(ka.camf, ka.H, x, y, uc, vc, lens, px, py, o, d);
      }
      depth = ka.max_depth;
      nstk = 0;
      in_path = true;
    }

    YK_STAMP(1);
    if (kCount && (ka.flags & kFlagTrace) && in_path) trace_ray(ka, slot, ka.max_depth - depth, o, d);

    // ---- closest hit (hittable_list.hpp:32-58 over sphere.hpp:25-48, in float)
    const bool alive = in_path && depth != 0;
    float T = INFINITY;
    int hid = -1;
    if (alive) {
      ++n_seg;
      const float a = ykf::len2(d);
      const float onorm = fmaxf(fabsf(o.x), fmaxf(fabsf(o.y), fabsf(o.z)));
      // the tree serves the rays its bound is proven for: |d|^2 in [2^-60, 2^60],
      // origin within origin_bound (< 0: the scene is outside the proven scale); the rest scan
      bool linear = (ka.flags & kFlagLinearScan) || !(a >= 0x1p-60f && a <= 0x1p60f) ||
                    !((double)onorm <= ka.origin_bound);
      if (!linear) {
        const float s = __builtin_sqrtf(a) * ykbvh::kF32Cone;  // the cone's slope (>= kF32Cone |d|)
        const float tmin_lo = tmin * (1.0f - 0x1p-17f);
        float ustar_f = INFINITY;  // T (1 + 2^-18): every box that may hold a root <= T passes
        f2 inx, ncx, jfx, fcx, iny, ncy, jfy, fcy, inz, ncz, jfz, fcz;
        cone_axis(d.x, o.x, s, inx, ncx, jfx, fcx);
        cone_axis(d.y, o.y, s, iny, ncy, jfy, fcy);
        cone_axis(d.z, o.z, s, inz, ncz, jfz, fcz);
        // the (near x4, far x4) plane quads of the ray's direction signs inside a WideNode
        const char* const px = nodes + (d.x < 0.0f ? 16u : 0u);
        const char* const py = nodes + 48u + (d.y < 0.0f ? 16u : 0u);
        const char* const pz = nodes + 96u + (d.z < 0.0f ? 16u : 0u);
        // A slow axis (|d| < s, the cone opens both ways along it) has no far bound, but the cone
        // still enters a box that lies against the direction of travel only after its far-side
        // plane: o + (d - s sign d) t reaches it at t = (plane - o) / (d - s sign d) > 0, a lower
        // bound like a near distance (same FMA form and error).  Without it, a
        // ray grazing a field of boxes enters every box under its path.  One slow axis per ray
        // gets the bound (y, then x, then z); the others keep L = -inf.
#if YK_SLAB_PAIRS_F32
        f2 jl2 = {0.0f, -INFINITY};  // the (jl, cl) pair
#else
        f2 jl2 = {0.0f, 0.0f}, cl2 = {-INFINITY, -INFINITY};
#endif
        const char* pl = px + 16;
        {
          const float slow = s * kF32SlowAt;
          const float dk[3] = {d.z, d.x, d.y}, ok[3] = {o.z, o.x, o.y};
          const char* const pk[3] = {pz, px, py};
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            if (fabsf(dk[k]) < slow) {
              const float jl = __builtin_amdgcn_rcpf(dk[k] - (dk[k] < 0.0f ? -s : s));
#if YK_SLAB_PAIRS_F32
              jl2 = f2{jl, -(ok[k] * jl)};  // (jl, cl), read by op_sel
#else
              jl2 = f2{jl, jl};
              cl2 = f2{-(ok[k] * jl), -(ok[k] * jl)};
#endif
              pl = pk[k] + 16;
            }
          }
        }
        // U*: proven upper bound of the minimum root (culls with ustar_f = U* (1 + 2^-18)); the
        // candidate list (tuple index, lower bound) as in the FP64 kernel, nc = 5 on overflow
        const float ia = __builtin_amdgcn_rcpf(a);  // a in [2^-60, 2^60] here
        float ustar = INFINITY;
        uint32_t nc = 0, c0 = 0, c1 = 0, c2 = 0, c3 = 0;
        float l0 = 0, l1 = 0, l2 = 0, l3 = 0;
        uint32_t overflow = 0;  // a VGPR, not a lane-mask bool (see the FP64 kernel)
        int32_t node = ka.bvh_root;
        int32_t* top = stk;
        const int32_t* const stk_cap = stk + ka.stack_cap * kBlk;
        for (;;) {
          if (node >= 0) {
            if (kCount) ++n_node;
            YK_STAMP_NODE_ITERATION(lane);
            // the FP64 kernel's visit (same planes, margins and visit order), the cone's operands
            const f4 qnx = *(const f4*)(px + node), qfx = *(const f4*)(px + node + 16);
            const f4 qny = *(const f4*)(py + node), qfy = *(const f4*)(py + node + 16);
            const f4 qnz = *(const f4*)(pz + node), qfz = *(const f4*)(pz + node + 16);
            const int4 ch = *(const int4*)(nodes + node + 144);
            bool hk[4];
#if YK_SLAB_PAIRS_F32
            const f2 nx[2] = {slab_fma(qnx.xy, inx), slab_fma(qnx.zw, inx)};
            const f2 fx[2] = {slab_fma(qfx.xy, jfx), slab_fma(qfx.zw, jfx)};
            const f2 ny[2] = {slab_fma(qny.xy, iny), slab_fma(qny.zw, iny)};
            const f2 fy[2] = {slab_fma(qfy.xy, jfy), slab_fma(qfy.zw, jfy)};
            const f2 nz[2] = {slab_fma(qnz.xy, inz), slab_fma(qnz.zw, inz)};
            const f2 fz[2] = {slab_fma(qfz.xy, jfz), slab_fma(qfz.zw, jfz)};
            const f4 qsl = *(const f4*)(pl + node);
            const f2 sl[2] = {slab_fma(qsl.xy, jl2), slab_fma(qsl.zw, jl2)};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const float tn = slab_max3(slab_max3(nx[k >> 1][k & 1], ny[k >> 1][k & 1], nz[k >> 1][k & 1]),
                                         sl[k >> 1][k & 1], tmin_lo);
              const float tf = slab_min(slab_min3(fx[k >> 1][k & 1], fy[k >> 1][k & 1], fz[k >> 1][k & 1]), ustar_f);
              hk[k] = tn <= tf;
            }
#else
            const f4 qsl = *(const f4*)(pl + node);
            const f2 nx[2] = {__builtin_elementwise_fma(qnx.xy, inx, ncx), __builtin_elementwise_fma(qnx.zw, inx, ncx)};
            const f2 fx[2] = {__builtin_elementwise_fma(qfx.xy, jfx, fcx), __builtin_elementwise_fma(qfx.zw, jfx, fcx)};
            const f2 ny[2] = {__builtin_elementwise_fma(qny.xy, iny, ncy), __builtin_elementwise_fma(qny.zw, iny, ncy)};
            const f2 fy[2] = {__builtin_elementwise_fma(qfy.xy, jfy, fcy), __builtin_elementwise_fma(qfy.zw, jfy, fcy)};
            const f2 nz[2] = {__builtin_elementwise_fma(qnz.xy, inz, ncz), __builtin_elementwise_fma(qnz.zw, inz, ncz)};
            const f2 fz[2] = {__builtin_elementwise_fma(qfz.xy, jfz, fcz), __builtin_elementwise_fma(qfz.zw, jfz, fcz)};
            const f2 sl[2] = {__builtin_elementwise_fma(qsl.xy, jl2, cl2), __builtin_elementwise_fma(qsl.zw, jl2, cl2)};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              // (a chain: two v_max3)
              const float tn = fmaxf(fmaxf(fmaxf(fmaxf(nx[k >> 1][k & 1], ny[k >> 1][k & 1]), nz[k >> 1][k & 1]),
                                           sl[k >> 1][k & 1]), tmin_lo);
              const float tf = fminf(fminf(fminf(fx[k >> 1][k & 1], fy[k >> 1][k & 1]), fz[k >> 1][k & 1]), ustar_f);
              hk[k] = tn <= tf;
            }
#endif
            asm volatile("" ::"v"(ch.x), "v"(ch.y), "v"(ch.z), "v"(ch.w));
            if (hk[0] || hk[1] || hk[2] || hk[3]) {
              node = hk[3] ? ch.w : (hk[2] ? ch.z : (hk[1] ? ch.y : ch.x));
              *top = ch.x;
              top += (hk[0] && (hk[1] || hk[2] || hk[3])) ? kBlk : 0;
              *top = ch.y;
              top += (hk[1] && (hk[2] || hk[3])) ? kBlk : 0;
              *top = ch.z;
              top += (hk[2] && hk[3]) ? kBlk : 0;
              if (top > stk_cap) {  // stack full: abandon, the linear scan decides
                overflow = 1;
                top = stk;
                node = ykbvh::kEmptyLeaf;
              }
              continue;
            }
            if (top == stk) {  // as in the FP64 kernel
              node = ykbvh::kEmptyLeaf;
            } else {
              top -= kBlk;
              node = *top;
            }
            continue;
          } else {
            YK_STAMP(2);
            const uint32_t v = ~(uint32_t)node, first = v >> 4, cnt = v & 15u;
            // bound-then-evaluate, as in the FP64 kernel: the exact discriminant decides disc < 0,
            // the root gets bounds only, and the survivors' exact roots are evaluated after the
            // traversal, with the lanes converged
            // (the FP32 tree has at most two spheres per leaf: the loop unrolled, without a loop
            // counter or latch; FP32 512 spp: -2.7%)
#pragma unroll
            for (uint32_t k = 0; k < kLeafCapF32; ++k) {
              if (k >= cnt) break;
              const float4 sg = leaf_geo[first + k];
              const uint32_t id = leaf_ids[first + k];
              asm volatile("" ::"v"(id));
              if (kCount) ++n_test;
              const ykf::v3 oc = {o.x - sg.x, o.y - sg.y, o.z - sg.z};
              const float hb = ykf::dot(oc, d);
              const float c = ykf::len2(oc) - sg.w;
              const float disc = hb * hb - a * c;
              if (disc < 0) continue;
              YK_STAMP_DISC_POS();
              float lb, ub;
              if (!f32_root_bounds(hb, disc, ia, tmin, lb, ub)) continue;
              if (!(lb <= ustar)) continue;
              if (ub < ustar) {
                ustar = ub;
                ustar_f = ub * (1.0f + 0x1p-18f);
              }
              if (nc == 4) {  // compact: drop entries the new bound has excluded
                uint32_t m2 = 0;
                uint32_t d0 = c0, d1 = c1, d2 = c2, d3 = c3;
                float e0 = l0, e1 = l1, e2 = l2, e3 = l3;
                if (e0 <= ustar) { YK_CAND_SET(m2, d0, e0); ++m2; }
                if (e1 <= ustar) { YK_CAND_SET(m2, d1, e1); ++m2; }
                if (e2 <= ustar) { YK_CAND_SET(m2, d2, e2); ++m2; }
                if (e3 <= ustar) { YK_CAND_SET(m2, d3, e3); ++m2; }
                nc = m2;
              }
              if (nc < 4) {
                c3 = c2, l3 = l2, c2 = c1, l2 = l1, c1 = c0, l1 = l0;
                c0 = id, l0 = lb;
                ++nc;
              } else {
                nc = 5;  // the list is full: the ordered scan decides
              }
            }
            YK_STAMP(6);
          }
          if (top == stk) break;
          top -= kBlk;
          node = *top;
        }
        YK_STAMP(2);
        if (overflow != 0) linear = true;
        if (nc > 4) linear = true;
        if (!linear) {
          // the survivors' exact roots: the minimum wins, an exact tie goes to the later tuple
          // index (hittable_list.hpp:36-43); a candidate whose lower bound exceeds the final U*
          // cannot be the minimum
#define YK_F32_EVAL(C, L)                                                       \
  if ((L) <= ustar) {                                                           \
    float r = 0.0f;                                                             \
    const int res = f32_root(geo_f[C], o, d, a, ra, a_ok, tmin, r, n_nit);      \
    if (kCount && res > 0) ++n_sqrt, ++n_ncall;                                 \
    if (res == 2 && (r < T || (r == T && (int)(C) > hid))) T = r, hid = (int)(C); \
  }
          const bool a_ok = ykf::div_range(a);
          const float ra = ykf::rcp_refined(a);
          if (nc > 0) YK_F32_EVAL(c0, l0)
          if (nc > 1) YK_F32_EVAL(c1, l1)
          if (nc > 2) YK_F32_EVAL(c2, l2)
          if (nc > 3) YK_F32_EVAL(c3, l3)
#undef YK_F32_EVAL
        }
      }
      if (linear) {  // the reference's ordered scan in tuple order (wave-uniform scalar loads)
        ++n_lin;
        T = INFINITY;
        hid = -1;
        for (uint32_t i = 0; i < ka.nspheres; ++i) {
          const float4 sg = ka.geo_f[i];
          if (kCount) ++n_test;
          const ykf::v3 oc = {o.x - sg.x, o.y - sg.y, o.z - sg.z};
          const float hb = ykf::dot(oc, d);
          const float c = ykf::len2(oc) - sg.w;
          const float disc = hb * hb - a * c;
          if (disc < 0) continue;
          if (kCount) ++n_sqrt, ++n_ncall;
          const float sq = ykf::nsqrt(disc, n_nit);
          float root = (-hb - sq) / a;
          if (root < tmin || T < root) {
            root = (-hb + sq) / a;
            if (root < tmin || T < root) continue;
          }
          T = root;
          hid = (int)i;
        }
      }
    }

    YK_STAMP(3);
    // ---- shade (raytracer.hpp:25-36, material.hpp), material-uniform as in the FP64 kernel: one
    //      block of canonicals (float: one word each) for lambertian's vec3::random (3), the fuzzed
    //      metal's factor and vector (4) and the dielectric's uniform (1, drawn speculatively and
    //      given back on total internal reflection); one normalisation; one second square root
    //      (the fuzzed metal's |vector|, the dielectric's sin(theta)).  Each lane's own operations
    //      and their order are the reference's render<float>.
    bool ended = in_path && !alive;
    double L_r = 0, L_g = 0, L_b = 0;
    if (alive) {
      SphereMat m{};
      ykf::v3 p{0, 0, 0}, nrm{0, 0, 0};
      bool front = false;
      if (hid >= 0) {
        const float4 sg = geo_f[hid];
        m = mat[hid];
        p = ykf::add(o, ykf::mul(d, T));  // ray::at
        const ykf::v3 outward = ykf::divs_fast_r(ykf::sub(p, ykf::v3{sg.x, sg.y, sg.z}), (float)m.radius, m.inv_rf);
        front = ykf::dot(d, outward) < 0;
        nrm = front ? outward : ykf::neg(outward);
      }
      const bool lamb = hid >= 0 && m.kind == YK_MATERIAL_LAMBERTIAN;
      const bool fuzzy = hid >= 0 && m.kind == YK_MATERIAL_METAL && m.fuzz > 0;
      const bool diel = hid >= 0 && m.kind == YK_MATERIAL_DIELECTRIC;
      const bool spec = diel && ykd::rng_can_speculate(g);
      const Gen saved = g;  // the dielectric's engine before its speculative draw
      const uint32_t ncan = lamb ? 3u : (fuzzy ? 4u : (spec ? 1u : 0u));
      float c0 = 0, c1 = 0, c2 = 0, c3 = 0;
      if (__ballot(ncan > 0 && !ykd::rng_lazy_ok(g, ncan)) == 0) {
        if (ncan > 0) c0 = ykf::canonical<true>(g);
        if (ncan > 1) c1 = ykf::canonical<true>(g);
        if (ncan > 2) c2 = ykf::canonical<true>(g);
        if (ncan > 3) c3 = ykf::canonical<true>(g);
      } else {
        if (ncan > 0) c0 = ykf::canonical(g);
        if (ncan > 1) c1 = ykf::canonical(g);
        if (ncan > 2) c2 = ykf::canonical(g);
        if (ncan > 3) c3 = ykf::canonical(g);
      }
      // lambertian: vec3::random(-1, 1), x then y then z; fuzzed metal: the length factor first
      const ykf::v3 rv = lamb ? ykf::v3{ykf::uniform_of(c0, -1.0f, 1.0f), ykf::uniform_of(c1, -1.0f, 1.0f),
                                        ykf::uniform_of(c2, -1.0f, 1.0f)}
                              : ykf::v3{ykf::uniform_of(c1, -1.0f, 1.0f), ykf::uniform_of(c2, -1.0f, 1.0f),
                                        ykf::uniform_of(c3, -1.0f, 1.0f)};
      const ykf::v3 vn = lamb ? rv : d;
      if (kCount) ++n_ncall;
      const ykf::v3 un = ykf::divs_fast(vn, ykf::nsqrt(ykf::len2(vn), n_nit));
      float ct = 0;  // dielectric: cos(theta) = min(dot(-unit, n), 1)
      if (diel) {
        ct = ykf::dot(ykf::neg(un), nrm);
        if (!(ct < 1.0f)) ct = 1.0f;
      }
      float sq2 = 0;  // fuzzed metal: |random vector|; dielectric: sin(theta)
      if (fuzzy || diel) sq2 = ykf::nsqrt(fuzzy ? ykf::len2(rv) : 1.0f - ct * ct, n_nit);
      if (hid < 0) {
        // sky: normalized(dir).y is a float; + 1.0 and the lerp are double (raytracer.hpp:35-36)
        const double t = ((double)un.y + 1.0) / 2;
        L_r = (1.0 - t) * 1.0 + t * 0.5;
        L_g = (1.0 - t) * 1.0 + t * 0.7;
        L_b = (1.0 - t) * 1.0 + t * 1.0;
        ended = true;
      } else {
        bool scattered = true, push = true;
        ykf::v3 nd;
        if (m.kind == YK_MATERIAL_LAMBERTIAN) {
          nd = ykf::add(nrm, un);
          if (ykf::near_zero(nd)) nd = nrm;
        } else if (m.kind == YK_MATERIAL_METAL) {
          nd = ykf::reflect(un, nrm);
          if (fuzzy) {
            const float k = ykf::uniform_of(c0, 0.01f, 0.99f);
            const ykf::v3 ru = ykf::divs_fast(rv, sq2);
            nd = ykf::add(nd, ykf::mul(ykf::mul(ru, k), (float)m.fuzz));
          }
          scattered = ykf::dot(nd, nrm) > 0;
        } else {  // dielectric extension, in float
          push = false;
          const float ior = (float)m.ior;
          const float ratio = front ? (1.0f / ior) : ior;
          const bool cannot = ratio * sq2 > 1.0f;
          float u = 0;
          if (cannot) {
            if (spec) g = saved;  // `cannot || ...` never draws: give the word back
          } else {
            u = spec ? c0 : ykf::canonical(g);
          }
          if (cannot || ykf::reflectance(ct, ratio) > u) {
            nd = ykf::reflect(un, nrm);
          } else {
            const ykf::v3 perp = ykf::mul(ykf::add(un, ykf::mul(nrm, ct)), ratio);
            const float pl = 1.0f - ykf::len2(perp);
            nd = ykf::add(perp, ykf::mul(nrm, -ykf::nsqrt(pl < 0 ? -pl : pl, n_nit)));
          }
        }
        if (!scattered) {
          ended = true;
        } else {
          if (push) {
            if (nstk >= kStackRegs) id_spill[nstk - kStackRegs] = (uint16_t)(st3 >> 16);
            st3 = (st3 << 16) | (st2 >> 16);
            st2 = (st2 << 16) | (st1 >> 16);
            st1 = (st1 << 16) | (st0 >> 16);
            st0 = (st0 << 16) | (uint32_t)hid;
            ++nstk;
          }
          o = p;
          d = nd;
          --depth;
        }
      }
    }

    YK_STAMP(4);
    if (ended) {
      // attenuation (double albedo) back to front, as in FP64 (raytracer.hpp:31)
      while (nstk > 0) {
        const uint32_t id = st0 & 0xffffu;
        st0 = (st0 >> 16) | (st1 << 16);
        st1 = (st1 >> 16) | (st2 << 16);
        st2 = (st2 >> 16) | (st3 << 16);
        st3 = (st3 >> 16) | (nstk > kStackRegs ? ((uint32_t)id_spill[nstk - kStackRegs - 1] << 16) : 0u);
        --nstk;
        const SphereMat m = mat[id];
        L_r = m.ar * L_r;
        L_g = m.ag * L_g;
        L_b = m.ab * L_b;
      }
      if (ykd::mt_used_fallback(g)) ++n_fb;
      if (kCount) n_words += ykd::rng_words(g), n_twist += ykd::rng_twists(g);
      colour_store(ka.col, slot, L_r, L_g, L_b);
      in_path = false;
    }
    YK_STAMP(5);
  }
  YK_CLOCK_END(ka);
  YK_STAMPS_END(ka.counters, lane);
  if (kCount) {
    atomicAdd(&ka.counters[0], (unsigned long long)n_seg);
    atomicAdd(&ka.counters[1], (unsigned long long)n_test);
    atomicAdd(&ka.counters[2], (unsigned long long)n_sqrt);
    atomicAdd(&ka.counters[4], (unsigned long long)n_node);
    atomicAdd(&ka.counters[5], (unsigned long long)n_lin);
    atomicAdd(&ka.counters[6], (unsigned long long)n_ncall);
    atomicAdd(&ka.counters[7], (unsigned long long)n_nit);
    atomicAdd(&ka.counters[29], (unsigned long long)n_words);
    atomicAdd(&ka.counters[30], (unsigned long long)n_swords);
    atomicAdd(&ka.counters[31], (unsigned long long)n_twist);
  }
  if (n_fb) atomicAdd(&ka.counters[3], (unsigned long long)n_fb);
}

// The FP32 instance for (scene in LDS, kMode)
RenderKernel f32_kernel(bool lds, int mode) {
  static const RenderKernel k[8] = {yk_render_f32<false, 0>, yk_render_f32<false, 1>, yk_render_f32<false, 4>,
                                    yk_render_f32<false, 5>, yk_render_f32<true, 0>,  yk_render_f32<true, 1>,
                                    yk_render_f32<true, 4>,  yk_render_f32<true, 5>};
  return k[(lds ? 4 : 0) + ((mode & 1) | ((mode & 4) >> 1))];
}

#endif  // YK_SPLIT != 1

// ykgpu_math_sqrt_f32: the FP32 path's math::sqrt<float> on a buffer (diagnostic).
__global__ __launch_bounds__(256) void yk_math_sqrt_f32(const float* in, float* out, uint64_t n) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t it = 0;
  if (i < n) out[i] = ykf::nsqrt(in[i], it);
}

}  // namespace

#if YK_SPLIT == 2
// the FP32 unit's instances, for the main unit's f32_kernel()
extern "C" const void* yk_split_f32_kernel(bool lds, int mode) { return (const void*)f32_kernel(lds, mode); }
#else
#if YK_SPLIT == 1
extern "C" const void* yk_split_f32_kernel(bool lds, int mode);  // ykgpu_render_f32.o
namespace {
RenderKernel f32_kernel(bool lds, int mode) { return (RenderKernel)yk_split_f32_kernel(lds, mode); }
}  // namespace
#endif

// =========================================================================================
// C-ABI
// =========================================================================================
// A BVH on the device: the FP64 kernel's (boxes grown for the exact test's rounding, DESIGN.md
// §4) or the FP32 kernel's (grown for render<float>'s sphere test, §4.1), with its LDS layout
// [nodes][leaf geometry][leaf ids][traversal stacks] and the persistent grid it leaves room for.
struct DevTree {
  DevNode* nodes = nullptr;
  void* leaf_geo = nullptr;      // SphereGeo (FP64) or float4 (FP32), in leaf order
  uint32_t* leaf_ids = nullptr;  // leaf slot → tuple index
  int32_t root = 0;              // root code (byte offset of the root node, or a leaf code)
  uint32_t depth = 0, n_nodes = 0;
  double origin_bound = 0;  // |o|_inf beyond which a ray takes the linear scan (< 0: every ray)
  uint32_t geo_off = 0, ids_off = 0;  // leaf geometry and ids in LDS, after the nodes
  size_t bytes = 0;                   // device bytes of nodes, leaf geometry and ids
  // LDS plan per kernel shape: [0] kBlock threads (mt19937 instances), [1] kBlockX128 (xor128)
  struct Plan {
    bool in_lds = false;
    uint32_t lds_bytes = 0, stack_off = 0, stack_cap = 0, stack_entries = 0;
    bool stack_check = true;  // the kernel checks the stack top against stack_cap
    uint32_t tgeo_off = 0, mat_off = 0;  // shading tables in LDS (FP64 kernel), 0: none
    int grid = 0;                        // persistent blocks: occupancy x CUs
  } plan[2];
  void release() {
    (void)hipFree(nodes);
    (void)hipFree(leaf_geo);
    (void)hipFree(leaf_ids);
    nodes = nullptr;
    leaf_geo = nullptr;
    leaf_ids = nullptr;
    bytes = 0;
  }
};

struct ykgpu_context {
  int device = 0;
  int cus = 0;
  DevTree t64, t32;  // the FP64 and FP32 kernels' trees over the current scene
  size_t scratch_lanes = 0;
  char* d_warm = nullptr;  // warm-up ring: a StartRec (FP64) or StartRecF (FP32) per sample slot
  uint4* d_retry = nullptr;  // the FP64 warm-ups' lens-retry rings: retry_cap x 48 B per wave
  size_t retry_cap = 0;
  double* d_col = nullptr;     // sample colours of one launch (kColStride doubles per slot)
  double* d_acc = nullptr;     // running per-pixel sums between launches
  size_t col_cap = 0, acc_cap = 0;
  uint32_t* d_order = nullptr;  // processing slot → tile pixel, for (order_w, order_rows)
  uint32_t order_w = 0, order_rows = 0, order_slots = 0, order_stride = 0, order_mode = 0;
  size_t warm_cap = 0;
  hipStream_t stream = nullptr;
  hipStream_t aux = nullptr;  // the MT warm-ups run here, beside the render launches
  hipStream_t red = nullptr;  // the ordered reduces run here, beside the next render launch
  hipStream_t alt = nullptr;  // odd render launches: a launch starts while the previous drains
  hipStream_t ren = nullptr;  // even render launches (alt and ren: the device's top stream priority)
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  std::vector<hipEvent_t> lev;  // per launch: warm-up start, render start, reduce start, end
  uint32_t lev_used = 0;
  // Cross-call pipelining (launch()): the previous call's per-launch events and ring geometry, and
  // a global launch counter that numbers the ring slots, the scratch parity and the render
  // stream across calls
  std::vector<hipEvent_t> lev_prev;
  uint32_t lev_prev_used = 0;  // (events of the previous call in lev_prev: YKGPU_TIMELINE prints them)
  uint32_t prev_n = 0;
  // per global launch number g (mod kDepRing): its render's end and its reduce's end, the events a
  // later launch that reuses its start-record or colour buffer waits for, whichever call it was in
  std::vector<hipEvent_t> gev;
  // launches enqueued back to back with the current ring geometry (prev_geom), over calls: a call
  // overlaps the ones before it only when the last max(ring depths) launches had its geometry
  uint64_t run_len = 0;
  // the previous call's ring and scratch geometry: a call overlaps it only when every field is
  // equal (launch() `ov`; equal slot offsets in every ring buffer and scratch slice)
  struct RingGeom {
    uint64_t nps = 0, K = 0, welem = 0, warm_ring = 0, col_ring = 0, lanes = 0, id_stride = 0;
    const void *warm = nullptr, *col = nullptr, *mt = nullptr, *ids = nullptr;
    bool operator==(const RingGeom& o) const {
      return nps == o.nps && K == o.K && welem == o.welem && warm_ring == o.warm_ring && col_ring == o.col_ring &&
             lanes == o.lanes && id_stride == o.id_stride && warm == o.warm && col == o.col && mt == o.mt &&
             ids == o.ids;
    }
  } prev_geom;
  uint64_t prev_shape = 0;  // (nps, kmax, precision, engine) of the previous call: launch() `inflight`
  bool prev_ok = false;
  bool prev_enqueued = false;  // the previous call's launches were all enqueued (its events exist)
  bool dirty = false;          // a call failed part-way: its enqueued work is not tracked
  uint64_t g_next = 0;
  SphereGeo* d_geo = nullptr;
  SphereMat* d_mat = nullptr;
  float4* d_geo_f = nullptr;  // FP32 geometry (cx, cy, cz, r*r in float), tuple order
  uint32_t nspheres = 0;
  yk_camera cam{};
  bool have_scene = false;
  uint32_t* d_counter = nullptr;        // sample-slot counters, one per launch of a call
  uint32_t counter_cap = 0;
  unsigned long long* d_clk = nullptr;  // shader-clock probes, 4 words per launch (YK_CLOCK_*)
  unsigned long long* d_stats = nullptr;  // kCounters counters
  uint32_t* d_mt = nullptr;            // grid*256*624 words
  uint16_t* d_ids = nullptr;            // grid*256*id_stride
  uint32_t id_stride = 0;
  size_t id_lanes = 0;
  uint8_t* d_rgb = nullptr;
  size_t rgb_cap = 0;
  double* d_sums = nullptr;
  size_t sums_cap = 0;
  yk_render_stats stats{};
  bool stats_pending = false;
  double* d_trace = nullptr;  // ykgpu_render_trace's buffers (only during that call)
  uint32_t* d_trace_counts = nullptr;
  uint32_t trace_cap = 0;
  std::chrono::steady_clock::time_point t0;
};

struct ykgpu_group {
  std::vector<ykgpu_context*> ctx;  // one per entry of the device list
  std::vector<uint8_t*> tile;       // each entry's RGB8 tile on its device
  std::vector<size_t> tile_cap;
  std::vector<yk_render_stats> st;  // the last render's, per entry
  yk_render_stats total{};          // ... and of the whole call
};

namespace {

// A/B knobs: environment overrides of the launch schedule, rings, grids and tree build that the
// A/B tools time (tools/abtime.py `lib@YKGPU_X=v`).  They exist only in variant builds
// (tools/build_def_variant.sh <name> -DYK_AB_KNOBS): in the product library ab_knob() is a
// constant nullptr, so nothing in a caller's environment changes the schedule or the tree.  The
// documented diagnostics YKGPU_TIMELINE and YKGPU_OVERLAP stay.
#ifdef YK_AB_KNOBS
const char* ab_knob(const char* name) { return std::getenv(name); }
#else
constexpr const char* ab_knob(const char*) { return nullptr; }
#endif

uint64_t host_row_y(const yk_render_params* p, uint32_t t) {
  const uint32_t L = p->row_band_log2;
  return (uint64_t)p->row_begin + ((((uint64_t)(t >> L)) * p->row_stride) << L) + (t & ((1u << L) - 1u));
}

// The tile's width: its column set's size, or the image width (col_count == 0)
uint32_t tile_width(const yk_render_params* p) { return p->col_count ? p->col_count : p->image_width; }
uint64_t host_col_x(const yk_render_params* p, uint32_t j) {
  if (!p->col_count) return j;
  const uint32_t L = p->col_band_log2;
  return (uint64_t)p->col_begin + ((((uint64_t)(j >> L)) * p->col_stride) << L) + (j & ((1u << L) - 1u));
}

// Magic numbers of fdiv (kernel side) for a divisor 1 <= d < 2^31
void fastdiv(uint32_t d, uint32_t& m, uint32_t& sh) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  sh = 31 + l;
  m = (uint32_t)(((1ull << sh) + d - 1) / d);
}

int check_params(const ykgpu_context* ctx, const yk_render_params* p) {
  if (!ctx || !p) return fail(YK_ERR_INVALID, "null context or params");
  if (!ctx->have_scene) return fail(YK_ERR_NO_SCENE, "ykgpu_set_scene was not called");
  if (!p->image_width || !p->image_height || !p->samples_per_pixel)
    return fail(YK_ERR_INVALID, "image_width, image_height and samples_per_pixel must be > 0");
  if (!p->row_count) return fail(YK_ERR_INVALID, "row_count must be > 0");
  if (!p->row_stride) return fail(YK_ERR_INVALID, "row_stride must be > 0");
  if (p->row_band_log2 > 10) return fail(YK_ERR_INVALID, "row_band_log2 must be <= 10");
  if (host_row_y(p, p->row_count - 1) >= p->image_height) return fail(YK_ERR_INVALID, "row range outside the image");
  if (p->col_count) {
    if (!p->col_stride) return fail(YK_ERR_INVALID, "col_stride must be > 0");
    if (p->col_band_log2 > 10) return fail(YK_ERR_INVALID, "col_band_log2 must be <= 10");
    if (host_col_x(p, p->col_count - 1) >= p->image_width) return fail(YK_ERR_INVALID, "column range outside the image");
  } else if (p->col_begin || p->col_stride || p->col_band_log2) {
    return fail(YK_ERR_INVALID, "col_count == 0 (every column) needs col_begin, col_stride, col_band_log2 == 0");
  }
  if ((uint64_t)p->row_count * tile_width(p) >= (1ull << 31))
    return fail(YK_ERR_INVALID, "tile larger than 2^31 pixels");
  if (p->precision != YK_PRECISION_FP64 && p->precision != YK_PRECISION_FP32)
    return fail(YK_ERR_UNSUPPORTED, "precision mode");
  if (p->rng != YK_RNG_MT19937 && p->rng != YK_RNG_XOR128) return fail(YK_ERR_UNSUPPORTED, "rng mode");
  if (p->seed_mode != YK_SEED_COUNTER && p->seed_mode != YK_SEED_RANDOM_DEVICE)
    return fail(YK_ERR_UNSUPPORTED, "seed mode");
  if (!(p->t_min >= 0)) return fail(YK_ERR_INVALID, "t_min must be >= 0");
  // the one-lane diagnostic exists only in the FP64 counting instance: anywhere else it would be
  // ignored and a profile reconciled against the one-lane model would read all-lane counters
  if ((p->flags & YK_FLAG_ONE_LANE) &&
      (!(p->flags & YK_FLAG_COUNT_WORK) || p->precision != YK_PRECISION_FP64))
    return fail(YK_ERR_INVALID, "YK_FLAG_ONE_LANE needs YK_FLAG_COUNT_WORK and FP64");
  return YK_OK;
}

// Waits for every stream of the context: before a buffer that an earlier call's kernels may still
// use is freed (with cross-call pipelining a call's first launches run beside the previous call's
// last ones, launch())
int quiesce(ykgpu_context* ctx) {
  for (hipStream_t s : {ctx->aux, ctx->red, ctx->ren, ctx->alt, ctx->stream}) YK_HIP(hipStreamSynchronize(s));
  return YK_OK;
}

int ensure_scratch(ykgpu_context* ctx, uint32_t max_depth, size_t lanes, bool need_mt) {
  // mt19937 fallback engines: 624 words per persistent lane (not needed by xor128)
  if (need_mt && (lanes > ctx->scratch_lanes || !ctx->d_mt)) {
    if (int rc = quiesce(ctx)) return rc;
    (void)hipFree(ctx->d_mt);
    ctx->d_mt = nullptr;
    ctx->scratch_lanes = 0;
    YK_HIP(hipMalloc(&ctx->d_mt, 2 * lanes * ykd::kMtN * sizeof(uint32_t)));  // two launches in flight
    ctx->scratch_lanes = lanes;
  }
  // attenuation-id spill: max_depth u16 per lane
  const uint32_t need = max_depth > kStackRegs ? max_depth : 1;
  if (need > ctx->id_stride || lanes > ctx->id_lanes || !ctx->d_ids) {
    if (int rc = quiesce(ctx)) return rc;
    if (ctx->d_ids) YK_HIP(hipFree(ctx->d_ids));
    ctx->d_ids = nullptr;
    ctx->id_stride = 0;
    ctx->id_lanes = 0;
    YK_HIP(hipMalloc(&ctx->d_ids, 2 * lanes * need * sizeof(uint16_t)));
    ctx->id_stride = need;
    ctx->id_lanes = lanes;
  }
  return YK_OK;
}

#ifndef YK_LAUNCH_MB
#define YK_LAUNCH_MB 8192
#endif
// colour records of one launch at most: bounds a launch's slots for very large tiles (kmax in
// launch())
constexpr uint64_t kLaunchBytes = (uint64_t)YK_LAUNCH_MB << 20;
// the render kernel addresses a slot's start record as 4 * slot uint4s (FP32: 3) in 32-bit
// arithmetic
static_assert(kLaunchBytes / (8 * kColStride) * 4 < (1ull << 32), "4 * slot must fit 32 bits");
// samples per pixel per launch at most: many mid-sized launches beat a few big ones, because the
// launches alternate between two streams and each one's drain overlaps the next one's start
// (round 1, 1920x1080x512 259.5 -> 254.0 ms at 64 spp/launch; with the render
// streams at top priority, bench 205.5 ms at 64, 199.6 at 32, 199.8 at 24, 206.3 at 16)
#ifndef YK_LAUNCH_SPP
#define YK_LAUNCH_SPP 32
#endif
constexpr uint32_t kLaunchSpp = YK_LAUNCH_SPP;
// ... and for a call enqueued while the previous one still runs (launch() `inflight`): its launches
// need no ramp and overlap the calls around them, so the per-launch handover is what is left, and
// half as many launches pay it (frame: 8 of 64 instead of 16 of 32: bench -1.7%); a synced call
// keeps kLaunchSpp (64 there cost it 2%: the 64-spp warm-up under the ramp's 32-spp render and a
// longer last launch alone on the device, profiles/r06_ab/shade/).  The rings hold the larger
// launch in both, so a synced call and the in-flight calls after it share one ring geometry.
#ifndef YK_LAUNCH_SPP_OV
#define YK_LAUNCH_SPP_OV 64
#endif
constexpr uint32_t kLaunchSppOv = YK_LAUNCH_SPP_OV;
// ... or spp / kLaunchesPerCall when that is more (a long call: launch())
#ifndef YK_LAUNCHES_PER_CALL
#define YK_LAUNCHES_PER_CALL 32
#endif
constexpr uint32_t kLaunchesPerCall = YK_LAUNCHES_PER_CALL;
// ... and launches of about kLaunchSlots sample slots when the tile is small: a launch has a fixed
// cost (the handover of every CU from its render workgroup to the next launch's, filled by seed
// walks: ~0.2 ms per launch), so a call is split into round(slots / kLaunchSlots)
// launches — the frame's 32-spp launches are 66M slots, and a tile's launches are as large (the
// 8-way tile of 1920x1080x512: 2 launches of 256 spp; with 2^25-slot launches, 4 of 128, its
// back-to-back calls cost 2% more per sample than the frame's, profiles/r06_ab/tiles/)
#ifndef YK_LAUNCH_SLOTS
#define YK_LAUNCH_SLOTS (1u << 26)
#endif
constexpr uint64_t kLaunchSlots = YK_LAUNCH_SLOTS;
// ... and of about kLaunchSlotsOv for an in-flight call (as kLaunchSppOv for the frame), never
// fewer than two launches where a synced call has two: the 4-way tile 38.73 -> 38.59 ms, the 2-way
// 76.73 -> 76.18, config 4's 8-way 153.78 -> 153.10, the 8-way unchanged (profiles/r06_ab/tiles/r06ae_*)
#ifndef YK_LAUNCH_SLOTS_OV
#define YK_LAUNCH_SLOTS_OV (1u << 27)
#endif
constexpr uint64_t kLaunchSlotsOv = YK_LAUNCH_SLOTS_OV;
// (A/B) an in-flight call of one launch keeps the rings' full depth, so consecutive one-launch calls
// overlap like the launches of one call, and the floor of two launches goes
#ifndef YK_INFLIGHT_DEEP
#define YK_INFLIGHT_DEEP 0
#endif
constexpr bool kInflightDeep = YK_INFLIGHT_DEEP != 0;
// global launch numbers whose dependency events (ykgpu_context::gev) are kept: more than any ring
// is deep
constexpr uint32_t kDepRing = 16;
// Under memory pressure (launch()): launches shrink down to this many sample slots before a call
// fails with YK_ERR_NOMEM, and the rings leave kMemReserve of the device free
constexpr uint64_t kMemFloorSlots = 1ull << 24;
constexpr size_t kMemReserve = (size_t)512 << 20;
// Start-record ring: the warm-ups run on ctx->aux, beside the render launches (their wave slots
// and VGPRs fit next to the render kernel's, and the render leaves most VALU issue slots idle),
// into a ring of min(launches, kWarmRingDepth) launch buffers (YKGPU_WARM_RING overrides); warm-up
// c waits for the render of launch c - ring.  Sized to the call: ring x slots x record (1920x1080
// at 32 spp per launch: 66M slots x 64 B = 4.2 GB per launch buffer).
#ifndef YK_WARM_RING
#define YK_WARM_RING 3
#endif
constexpr uint32_t kWarmRingDepth = YK_WARM_RING;
#ifndef YK_FIRST_LAUNCH
#define YK_FIRST_LAUNCH 4
#endif
constexpr uint32_t kFirstLaunch = YK_FIRST_LAUNCH;  // samples per pixel in the first launch
// ... and each next launch grows by this factor until kmax: 4, 8, 16, 32, 32, ... (1920x1080x512:
// 4 + 8 + 16 + 14 x 32 + 18 + 18 = 512 spp in 19 launches).  Before round 4: 8, 32, 32, ...; its second
// warm-up (32 spp of walks beside the first render) sometimes finished late and delayed every
// launch after it: 20 synced calls on one box spread 173.6-177.4 ms (max/min 1.022), against
// 173.6-174.6 (1.0059) with 4, 8, 16 (tools/variance_ab.py, profiles/r04_ab/variance/)
#ifndef YK_SCHED_GROW
#define YK_SCHED_GROW 2
#endif
constexpr uint32_t kSchedGrow = YK_SCHED_GROW;
// ... and by half from this many samples per pixel on (0: kSchedGrow throughout)
#ifndef YK_SCHED_SLOW
#define YK_SCHED_SLOW 0
#endif
constexpr uint32_t kSchedSlow = YK_SCHED_SLOW;
// ... and for a call enqueued while the previous one still runs (launch(): `inflight`): every
// launch at kmax (YK_FIRST_LAUNCH_OV 0; else that many samples per pixel first, growing by
// YK_SCHED_GROW_OV)
#ifndef YK_FIRST_LAUNCH_OV
#define YK_FIRST_LAUNCH_OV 0
#endif
#ifndef YK_SCHED_GROW_OV
#define YK_SCHED_GROW_OV 4
#endif
constexpr uint32_t kFirstLaunchOv = YK_FIRST_LAUNCH_OV, kSchedGrowOv = YK_SCHED_GROW_OV;
static_assert(YK_FIRST_LAUNCH >= 1 && YK_LAUNCH_SPP >= 1, "launch sizes must be >= 1 sample per pixel");
#ifndef YK_TILE
#define YK_TILE 8
#endif
constexpr uint32_t kTile = YK_TILE;  // processing blocks of kTile x kTile pixels (0: row-major)

// The processing order of a tile of W x rows pixels (kernel comment at kNoPixel).  A function of
// the geometry only, so it is built once per size and kept on the device.  Blocks hold 64 tile
// pixels; for a tile of every stride-th image row (the N-GPU split) they are widened and
// flattened so that a block still covers a roughly square patch of the IMAGE (stride 1: 8 x 8;
// 2: 16 x 4 tile rows = 16 x 8 image rows; 4: 16 x 4 = 16 x 16; 8: 32 x 2 = 32 x 16): the rays a
// wave starts together stay coherent (8 x 8 tile blocks of a 4-way tile, 8 x 32 image pixels,
// cost 17% more per sample, measured).
int ensure_order(ykgpu_context* ctx, uint32_t W, uint32_t rows, uint32_t stride) {
  // (A/B knob: YKGPU_ORDER=1 takes the block rows bottom-up)
  const char* oe = ab_knob("YKGPU_ORDER");
  const uint32_t mode = oe ? (uint32_t)std::atoi(oe) : 0u;
  if (ctx->d_order && ctx->order_w == W && ctx->order_rows == rows && ctx->order_stride == stride &&
      ctx->order_mode == mode)
    return YK_OK;
  std::vector<uint32_t> ord;
  if (kTile == 0) {
    ord.resize((size_t)W * rows);
    for (size_t i = 0; i < ord.size(); ++i) ord[i] = (uint32_t)i;
  } else {
    const uint32_t th = stride <= 1 ? kTile : (stride <= 4 ? std::max(1u, kTile / 2) : std::max(1u, kTile / 4));
    const uint32_t tw = kTile * kTile / th;
    const uint32_t bx = (W + tw - 1) / tw, by = (rows + th - 1) / th;
    ord.reserve((size_t)bx * by * tw * th);
    for (uint32_t jj = 0; jj < by; ++jj)
      for (uint32_t i = 0; i < bx; ++i)
        for (uint32_t k = 0; k < tw * th; ++k) {
          const uint32_t j = mode == 1 ? by - 1 - jj : jj;
          const uint32_t x = i * tw + k % tw, y = j * th + k / tw;
          ord.push_back(x < W && y < rows ? y * W + x : kNoPixel);
        }
  }
  if (int rc = quiesce(ctx)) return rc;
  (void)hipFree(ctx->d_order);
  ctx->d_order = nullptr;
  ctx->order_w = ctx->order_rows = ctx->order_slots = 0;
  YK_HIP(hipMalloc(&ctx->d_order, ord.size() * sizeof(uint32_t)));
  YK_HIP(hipMemcpy(ctx->d_order, ord.data(), ord.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  ctx->order_w = W;
  ctx->order_rows = rows;
  ctx->order_stride = stride;
  ctx->order_mode = mode;
  ctx->order_slots = (uint32_t)ord.size();
  return YK_OK;
}

// Render streams get the device's top priority (YKGPU_RENDER_PRIO=0: default priority, A/B): when
// a launch drains, the queued warm-up and reduce blocks would otherwise take the CUs it frees
// before the next launch's workgroups (one per CU, 768 threads and most of the LDS) fit.
hipError_t create_render_stream(hipStream_t* s) {
  int least = 0, greatest = 0;
  const char* e = ab_knob("YKGPU_RENDER_PRIO");
  if ((e && std::atoi(e) == 0) || hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess)
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  return hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
}

// Colour buffers in flight (YKGPU_COL_RING overrides): render c writes buffer c % ring and waits
// for the reduce of launch c - ring.  Two suffice: a reduce (~0.6 ms for 32 spp of 1920x1080)
// ends long before the render after next needs its buffer; rings of 2 / 3 / 4 time the same
// (bench 171.8 / 171.8 / 172.1 ms; config-4 rank tile 174.0 vs 173.6 ms, profiles/r04_ab/rings/)
// and 2 holds 4.2 GB less at the headline size (call_bytes 22.3 -> 18.1 GB)
#ifndef YK_COL_RING
#define YK_COL_RING 2
#endif
#ifndef YK_RED_PRIO
#define YK_RED_PRIO 0
#endif
uint32_t col_ring() {
  uint32_t r = YK_COL_RING;
  if (const char* e = ab_knob("YKGPU_COL_RING")) r = (uint32_t)std::max(2, std::min(8, std::atoi(e)));
  return r;
}

// Reduce grid: grid-stride over the slots, at most 4 blocks per CU (YKGPU_RED_BLOCKS overrides;
// 0 = one thread per slot), so a reduce never floods the CUs a render launch is about to take
uint32_t reduce_blocks(const ykgpu_context* ctx, uint32_t nps) {
  uint32_t cap = (uint32_t)ctx->cus * 4;
  if (const char* e = ab_knob("YKGPU_RED_BLOCKS")) cap = (uint32_t)std::max(0, std::atoi(e));
  const uint32_t full = (nps + 255) / 256;
  return cap ? std::max(1u, std::min(full, cap)) : full;
}

// Warm-up grid: grid-stride, at most `per_cu` blocks (one wave per SIMD each) per CU
// (YKGPU_WARM_PER_CU overrides).  The FP64 StartRec warm-up is close to the render's critical
// path and takes every idle issue slot it can (32; 16: neutral, 8: +1.8%); the FP32 one has
// slack, and each resident warm-up wave delays the latency-bound render waves it shares a SIMD
// with (512-spp FP32 A/B: 32 -> 205.2 ms, 4 -> 202.4, 3 -> 202.4, 2 -> 201.3)
// FP64 warm-up grid: blocks per CU (each thread walks n / grid slots, at least kWarmSlots)
#ifndef YK_WARM_PER_CU
#define YK_WARM_PER_CU 32
#endif
#ifndef YK_WARM_SLOTS
#define YK_WARM_SLOTS 4
#endif
constexpr uint32_t kWarmSlots = YK_WARM_SLOTS;
uint32_t warm_per_cu(bool f32) {
  uint32_t per_cu = f32 ? 2u : (uint32_t)YK_WARM_PER_CU;
  if (const char* e = ab_knob("YKGPU_WARM_PER_CU")) per_cu = (uint32_t)std::max(1, std::atoi(e));
  return per_cu;
}
// A warm-up's blocks for n slots, at most cap: each thread walks n / grid slots, at least
// kWarmSlots; with ilp walks per lane the grid is trimmed so that a thread's slot count is a
// multiple of ilp (no lane walks a chain for a slot it does not have, but in the last blocks)
#ifndef YK_WARM_TRIM
#define YK_WARM_TRIM 1
#endif
inline uint32_t warm_blocks_for(uint64_t n, uint64_t cap, uint32_t ilp) {
  uint64_t wb = std::min<uint64_t>((n + 256 * kWarmSlots - 1) / (256 * kWarmSlots), cap);
  if (YK_WARM_TRIM && ilp > 1 && wb > 0) {
    const uint64_t per = 256ull * ilp, it = (n + wb * per - 1) / (wb * per);
    wb = (n + per * it - 1) / (per * it);
  }
  return (uint32_t)wb;
}

int launch(ykgpu_context* ctx, const yk_render_params* p, uint8_t* rgb_dev, double* sums_dev,
           hipStream_t st) {
  const bool f32 = p->precision == YK_PRECISION_FP32;
  const bool x128 = p->rng == YK_RNG_XOR128;  // no warm-ups, no MT scratch
  const DevTree& tree = f32 ? ctx->t32 : ctx->t64;
  const DevTree::Plan& plan = tree.plan[x128 ? 1 : 0];
  const int grid = plan.grid, block = block_of(x128);
  int rc = ensure_scratch(ctx, p->max_depth, (size_t)grid * block, !x128);
  if (rc) return rc;
  // YK_SEED_RANDOM_DEVICE without a key: one from std::random_device per call (source.cpp:159)
  uint64_t seed_key = 0;
  if (p->seed_mode == YK_SEED_RANDOM_DEVICE) {
    seed_key = p->seed_key;
    if (!seed_key) {
      std::random_device rd;
      while (!seed_key) seed_key = ((uint64_t)rd() << 32) | rd();
    }
  }
  // image rows per tile row, for the shape of the processing blocks (bands of >= 8 rows: 1,
  // an 8 x 8 block stays inside one band)
  rc = ensure_order(ctx, tile_width(p), p->row_count,
                    p->row_count > 1 && p->row_band_log2 < 3 ? p->row_stride : 1);
  if (rc) return rc;
  // Launch schedule (samples per pixel per launch): kFirstLaunch (4), growing by kSchedGrow (2)
  // up to kmax (kLaunchSpp = 32, or more for a small tile), also capped by the colour budget (32 B
  // per sample slot, kLaunchBytes per launch); a short remainder is folded into the launches before
  // it (1920x1080x512: 4, 8, 16, 14 x 32, 18, 18 = 19 launches).  The first render waits only for
  // a 4-sample warm-up, and each next warm-up, twice the one before, finishes under the render
  // before it (see kSchedGrow).  Each launch ends with the tail of its longest paths (~0.1-0.2 ms
  // of partly idle CUs), but launches alternate between two streams, so that drain overlaps the
  // next launch: many
  // mid-sized launches beat a few large ones.  Independent of the image size, which matters
  // for the per-rank tiles of N GPUs.
  const uint32_t nps = ctx->order_slots;  // processing slots (>= pixels)
  const uint32_t spp = p->samples_per_pixel;
  // (slots of a launch stay below 2^31: the kernels' fdiv takes 31-bit numerators)
  // A launch of few pixels still gets enough slots to fill the persistent grid (16 per lane):
  // a thin row tile at high spp would otherwise run dozens of launches that each pay a ramp and
  // a drain.  Neither floor nor cap exceeds the colour budget or 2^31 slots.
  const uint64_t fill_spp = ((uint64_t)grid * block * 16 + nps - 1) / nps;
  uint64_t launch_slots = kLaunchSlots;  // (A/B knob: YKGPU_LAUNCH_SLOTS)
  if (const char* e = ab_knob("YKGPU_LAUNCH_SLOTS")) launch_slots = (uint64_t)std::max(1ll, std::atoll(e));
  auto launches_for = [&](uint64_t lslots) {
    return std::max<uint64_t>(1, ((uint64_t)nps * spp + lslots / 2) / lslots);
  };
  // (in flight: never fewer than two launches where a synced call has two — a one-launch call has
  // rings of one buffer and overlaps nothing: the 8-way tile 19.6 -> 25.5 ms, r06ad)
  const uint64_t call_launches = launches_for(launch_slots);
  const uint64_t call_launches_ov =
      kInflightDeep ? launches_for(std::max(launch_slots, kLaunchSlotsOv))
                    : std::max(std::min<uint64_t>(call_launches, 2), launches_for(std::max(launch_slots, kLaunchSlotsOv)));
  const uint64_t slot_spp = (spp + call_launches - 1) / call_launches;
  const uint64_t slot_spp_ov = (spp + call_launches_ov - 1) / call_launches_ov;
  // A long call takes longer launches: every launch pays a drain whose length is the longest path
  // of its last samples, and many launches per call buy nothing once there are ~32 (config 5,
  // 1920x1080x4096 at depth 200 on the glass scene: 32 spp per launch 1730 ms, 64 1631, 121 (the
  // colour budget) 1589, with a warm ring of 2 1610; config 3's 512 spp stay at 32, where 64
  // costs 5%; profiles/r04_ab/launch_size/).  The rings grow with the launch: config 5 holds
  // ~64 GB (3 x 2.07M x 121 x 64 B of start records, 2 x 2.07M x 121 x 32 B of colours).
  uint64_t launch_spp = std::max<uint64_t>(kLaunchSpp, spp / kLaunchesPerCall);
  if (const char* e = ab_knob("YKGPU_LAUNCH_SPP")) launch_spp = (uint64_t)std::max(1, std::atoi(e));  // (A/B)
  const uint64_t launch_spp_ov = std::max<uint64_t>(std::max<uint64_t>(kLaunchSppOv, launch_spp), spp / kLaunchesPerCall);
  auto ideal_for = [&](uint64_t lspp, uint64_t sspp) {
    return (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>({spp, kLaunchBytes / (8ull * kColStride * nps),
                               std::max<uint64_t>({lspp, fill_spp, sspp}), ((1ull << 31) - 1) / nps}));
  };
  // the rings' launch size (an in-flight call's launches) and a synced call's, <= it
  const uint32_t kideal = ideal_for(launch_spp_ov, slot_spp_ov), ksynced = ideal_for(launch_spp, slot_spp);
  // A device short of memory (other contexts, other processes) makes the call slower, not fatal:
  // the rings are sized for launches of kmax samples per pixel, and when the device cannot hold
  // them — free memory (hipMemGetInfo) plus what this context's rings already hold, or a
  // hipMalloc that fails anyway — kmax halves, down to launches of kMemFloorSlots sample slots,
  // before the call fails with YK_ERR_NOMEM (yk_render_stats.launch_spp / mem_shrinks report it).
  const uint32_t kfloor = (uint32_t)std::min<uint64_t>(kideal, std::max<uint64_t>(1, (kMemFloorSlots + nps - 1) / nps));
  uint32_t kmax = kideal, mem_shrinks = 0;
  auto shrink = [&]() {
    kmax = std::max(kfloor, kmax / 2);
    ++mem_shrinks;
  };
  // a buffer follows the call: grown when it is too small, and given back when the call needs
  // less than half of it (device_bytes then reports about what the call holds)
  auto grow = [&](auto*& ptr, size_t& cap, size_t need, size_t elem) -> int {
    if (need <= cap && 2 * need >= cap) return YK_OK;
    if (int q = quiesce(ctx)) return q;
    (void)hipFree(ptr);
    ptr = nullptr;
    cap = 0;
    YK_HIP(hipMalloc((void**)&ptr, need * elem));
    cap = need;
    return YK_OK;
  };
  std::vector<std::pair<uint32_t, uint32_t>> sched;  // (s0, samples)
  uint64_t shape = 0;
  bool inflight = false;
  uint32_t K = 0, nlaunch = 0, kWarmRing = 0, kColRing = 0;
  // start records (StartRec, FP32 StartRecF: each sample's whole start)
  const size_t welem = f32 ? sizeof(StartRecF) : sizeof(StartRec);
  // (diagnostic, timing only) YKGPU_ABL_WARM_FIRST=1: every launch's warm-up runs, and finishes,
  // before the first render: render_busy_ms then times the render kernels without the seed walks
  // beside them (same images)
  const bool warm_first = ab_knob("YKGPU_ABL_WARM_FIRST") != nullptr && !x128;
  for (;;) {
    // A call enqueued while the previous one still runs (back-to-back steps) starts its first
    // warm-ups under the previous call's last launches, so it needs no small first launch: every
    // launch at kmax — the frame is 16 launches of 32 (bench 8 steps: 172.4 ms per step with 4, 8,
    // 16, 32; 170.8 with 8, 32; 168.4 with 32, 32, ...; profiles/r04_ab/schedule/), the 8-way tile
    // of config 3 four of ~130 (23.1 ms per call starting at 32, 21.8 at 128; the 4-way tile 44.3
    // -> 43.0 ms starting at 64; profiles/r04_ab/tiles/)
    // (A/B knobs: YKGPU_FIRST_LAUNCH, YKGPU_SCHED_GROW and their _OV forms — the first launch's
    // samples per pixel and the factor each next launch grows by until kmax)
    // (only for a call of the previous one's shape, whose rings it can overlap: launch() `ov`)
    shape = ((uint64_t)nps << 24) ^ ((uint64_t)kmax << 2) ^ (f32 ? 2u : 0u) ^ (x128 ? 1u : 0u);
    inflight = false;
    if (ctx->prev_enqueued && ctx->prev_ok && !ctx->dirty && ctx->prev_shape == shape && ctx->prev_n > 0 &&
        ctx->lev.size() >= 6ull * ctx->prev_n)
      inflight = hipEventQuery(ctx->lev[6 * (ctx->prev_n - 1) + 5]) == hipErrorNotReady;
    // this call's largest launch: the rings' (kmax) in flight, a synced call's own below it
    const uint32_t kcap = inflight ? kmax : std::min(kmax, ksynced);
    uint32_t first_k = inflight ? (kFirstLaunchOv ? kFirstLaunchOv : kmax) : kFirstLaunch;
    uint32_t grow_k = inflight ? kSchedGrowOv : kSchedGrow;
    if (const char* e = ab_knob(inflight ? "YKGPU_FIRST_LAUNCH_OV" : "YKGPU_FIRST_LAUNCH"))
      first_k = (uint32_t)std::max(1, std::atoi(e));
    if (const char* e = ab_knob(inflight ? "YKGPU_SCHED_GROW_OV" : "YKGPU_SCHED_GROW"))
      grow_k = (uint32_t)std::max(2, std::atoi(e));
    sched.clear();
    // the ramp (first_k, growing by grow_k), then launches of kmax; a short tail launch, which would
    // pay its own drain, is folded into the launch before it, or that launch and the tail are split
    // into two equal launches when one would exceed kmax — so no launch exceeds kmax, and every call
    // of the same kmax places its launches in the rings alike (a back-to-back call overlaps the
    // call before it, synced or not).  Launches of exactly kmax also keep the warm-up's walks
    // aligned: at 32 spp its grid-stride is the pixel count, so a lane's four walks are four
    // samples of one pixel (their processing-order reads coincide; a 30- or 31-spp launch fetches
    // 1.7x the bytes per slot in the warm-up, profiles/r06_ab/pmc/)
    for (uint32_t s0 = 0, k = std::min(first_k, kcap); s0 < spp;) {
      uint32_t take = std::min(k, spp - s0);
      const uint32_t rest = spp - (s0 + take);
      if (rest > 0 && rest < std::max(1u, take / 4))
        take = spp - s0 <= kcap ? spp - s0 : (spp - s0 + 1) / 2;
      sched.emplace_back(s0, take);
      s0 += take;
      // past kSchedSlow spp the ramp grows by half: a warm-up twice its render's size no longer
      // hides under it (64-spp launches: the 64-spp warm-up under the 32-spp render cost the
      // synced call 2%, profiles/r06_ab/shade/r06z_*)
      k = std::min(kSchedSlow && k >= kSchedSlow ? k + k / 2 : grow_k * k, kcap);
    }
    // a launch buffer of the rings holds kmax samples per pixel (every launch fits: above)
    K = kmax;
    nlaunch = (uint32_t)sched.size();
    // rings as deep as kWarmRingDepth / col_ring() whatever the call's launch count (a call of two
    // launches reuses the buffers of the call before it, launch() `ov`); one buffer each for a
    // single-launch call
    kWarmRing = nlaunch > 1 || (kInflightDeep && inflight) ? kWarmRingDepth : 1;
    if (const char* e = ab_knob("YKGPU_WARM_RING"))  // (A/B) launch buffers in the ring
      kWarmRing = (uint32_t)std::min<uint64_t>(kDepRing - 1, (uint64_t)std::max(2, std::atoi(e)));
    if (warm_first) kWarmRing = nlaunch;
    // colour buffers: render c writes buffer c % ring and waits for the reduce of launch c - ring;
    // reduce c (stream red) overlaps the renders after it
    kColRing = nlaunch > 1 || (kInflightDeep && inflight) ? std::min(col_ring(), kDepRing - 1) : 1;
    const size_t need_warm = x128 ? 0 : (size_t)kWarmRing * nps * K * welem;
    const size_t need_col = (size_t)kColRing * nps * K * kColStride * sizeof(double);
    if (kmax > kfloor && (need_warm > ctx->warm_cap || need_col > ctx->col_cap * sizeof(double))) {
      // the rings must grow: does the device have room for them?
      size_t free_b = 0, total_b = 0;
      if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
        const size_t held = ctx->warm_cap + ctx->col_cap * sizeof(double);
        if (need_warm + need_col + kMemReserve > free_b + held) {
          shrink();
          continue;
        }
      }
    }
    rc = x128 ? YK_OK : grow(ctx->d_warm, ctx->warm_cap, need_warm, 1);
    if (!rc) rc = grow(ctx->d_col, ctx->col_cap, (size_t)kColRing * nps * K * kColStride, sizeof(double));
    if (rc == YK_ERR_NOMEM && kmax > kfloor) {
      (void)hipGetLastError();  // (the failed hipMalloc's error must not surface at a later launch)
      shrink();
      continue;
    }
    if (rc) return rc;
    break;
  }
  if (sched.size() > 1 && (rc = grow(ctx->d_acc, ctx->acc_cap, (size_t)nps * 3, sizeof(double)))) return rc;
  // The FP64 lens warm-ups of launches with at most kDeferSlots slots per warm-up wave draw their
  // lens retries after the walks (yk_mt_warmup_defer) from a ring per wave, sized to the largest
  // such launch (the frame's 32-spp launches: 640 records, 1.0 GB); longer launches run the
  // rejection loop in line (config 5's 121-spp launches: 7600 slots per wave, where the deferral
  // measured 0.7% slower)
  const bool lens_defer = kLensDefer && !x128 && !f32 && ctx->cam.lens_radius > 0;
  auto wave_slots = [&](uint64_t nl) {
    const uint64_t wb = warm_blocks_for(nl, (uint64_t)ctx->cus * warm_per_cu(false), kWalkIlp);
    return (nl + wb * 256 - 1) / (wb * 256) * 64;
  };
  uint32_t retry_cap = 0;  // records per wave
  if (lens_defer)
    for (const auto& l : sched)
      if (wave_slots((uint64_t)nps * l.second) <= kDeferSlots)
        retry_cap = std::max(retry_cap, retry_cap_for(wave_slots((uint64_t)nps * l.second)));
  // a call whose launches were shrunk for want of memory runs the rejection loop in line: the
  // shrink loop above budgets the start-record and colour rings only, so the plan it settled on
  // is the plan the call runs (no ring allocated afterwards out of the reserve it kept)
  if (mem_shrinks) retry_cap = 0;
#ifdef YK_RETRY_CAP_FORCE
  // (test variants, tests/test_gpu_robust.py): the ring's capacity forced so that its fallbacks
  // run — 64 records per wave fill up (the samples that find it full reach the render as kNoStart
  // starts it makes itself), 0 is the in-line loop a failed ring allocation falls back to
  if (retry_cap) retry_cap = YK_RETRY_CAP_FORCE;
#endif
  size_t retry_n = (size_t)ctx->cus * warm_per_cu(false) * 4u * retry_cap * 3u;
  if (retry_cap && (rc = grow(ctx->d_retry, ctx->retry_cap, retry_n, sizeof(uint4)))) {
    if (rc != YK_ERR_NOMEM) return rc;
    // a device short of memory runs the rejection loop in line instead (slower, never fatal)
    (void)hipGetLastError();
    retry_cap = 0;
    retry_n = 0;
  }
  KernelArgs ka;
  ka.cam = ctx->cam;
  ka.pad_a = 0;
  {
    const yk_camera& c = ctx->cam;
    for (int k = 0; k < 3; ++k) {
      ka.camf.origin[k] = (float)c.origin[k];
      ka.camf.llc[k] = (float)c.lower_left_corner[k];
      ka.camf.horizontal[k] = (float)c.horizontal[k];
      ka.camf.vertical[k] = (float)c.vertical[k];
      ka.camf.lens_u[k] = (float)c.lens_u[k];
      ka.camf.lens_v[k] = (float)c.lens_v[k];
      ka.camf.pad[k] = 0.0f;
    }
    ka.camf.lens_radius = (float)c.lens_radius;
    ka.camf.w = (float)p->image_width;  // unsigned → float (source.cpp:162, T = float)
    ka.camf.h = (float)p->image_height;
  }
  ka.W = p->image_width;
  ka.Wt = tile_width(p);
  ka.col_begin = p->col_count ? p->col_begin : 0;
  ka.col_stride = p->col_count ? p->col_stride : 1;
  ka.col_band = p->col_count ? p->col_band_log2 : 0;
  ka.H = p->image_height;
  ka.spp = p->samples_per_pixel;
  ka.max_depth = p->max_depth;
  ka.seed0 = p->seed0;
  ka.row_begin = p->row_begin;
  ka.row_count = p->row_count;
  ka.row_stride = p->row_stride;
  ka.band_log2 = p->row_band_log2;
  ka.nspheres = ctx->nspheres;
  ka.flags = p->flags;
  ka.id_stride = ctx->id_stride;
  ka.start = nullptr;
  ka.order = ctx->d_order;
  ka.t_min = p->t_min;
  ka.origin_bound = tree.origin_bound;
  ka.inv_w = 1.0 / (double)ka.W;
  ka.inv_h = 1.0 / (double)ka.H;
  ka.w_d = (double)ka.W;
  ka.h_d = (double)ka.H;
  ka.bvh_root = tree.root;
  ka.n_nodes = tree.n_nodes;
  ka.lds_geo_off = tree.geo_off;
  ka.lds_ids_off = tree.ids_off;
  ka.lds_tgeo_off = plan.tgeo_off;
  ka.lds_mat_off = plan.mat_off;
  ka.lds_stack_off = plan.stack_off;
  ka.stack_cap = plan.stack_cap;
  ka.nodes = tree.nodes;
  ka.leaf_geo = (const SphereGeo*)tree.leaf_geo;  // float4 records for the FP32 kernel
  ka.leaf_ids = tree.leaf_ids;
  ka.geo = ctx->d_geo;
  ka.mat = ctx->d_mat;
  ka.geo_f = ctx->d_geo_f;
  ka.seed_mode = p->seed_mode;
  ka.seed_key = seed_key;
  ka.pixel_counter = ctx->d_counter;

  ka.counters = ctx->d_stats;
  ka.trace = ctx->d_trace;
  ka.trace_counts = ctx->d_trace_counts;
  ka.trace_cap = ctx->trace_cap;
  ka.claim_tail = (uint32_t)grid * (uint32_t)(block / 64) * kClaim * kClaimTailFactor;
  if ((ka.flags & YK_FLAG_TRACE_RAYS) && !(ctx->d_trace && (ka.flags & YK_FLAG_COUNT_WORK)))
    return fail(YK_ERR_INVALID, "YK_FLAG_TRACE_RAYS is set by ykgpu_render_trace only");
  WarmArgs wa;
  wa.W = p->image_width;
  wa.Wt = ka.Wt;
  wa.col_begin = ka.col_begin;
  wa.col_stride = ka.col_stride;
  wa.col_band = ka.col_band;
  wa.spp = p->samples_per_pixel;
  wa.seed0 = p->seed0;
  wa.row_begin = p->row_begin;
  wa.row_stride = p->row_stride;
  wa.band_log2 = p->row_band_log2;
  wa.out = ctx->d_warm;
  wa.retry = retry_cap ? ctx->d_retry : nullptr;
  wa.retry_cap = retry_cap;
  wa.retry_pad = 0;
  wa.lens = ctx->cam.lens_radius > 0 ? 1u : 0u;
  wa.H = p->image_height;
  wa.cam = ctx->cam;
  wa.camf = ka.camf;
  wa.w_d = ka.w_d;
  wa.h_d = ka.h_d;
  wa.inv_w = ka.inv_w;
  wa.inv_h = ka.inv_h;
  wa.npix_slots = nps;
  fastdiv(nps, wa.nps_m, wa.nps_sh);
  fastdiv(ka.Wt, wa.w_m, wa.w_sh);
  wa.seed_mode = p->seed_mode;
  wa.seed_key = seed_key;
  wa.order = ctx->d_order;
  ka.npix_slots = nps;
  ka.nps_m = wa.nps_m;
  ka.nps_sh = wa.nps_sh;
  ka.w_m = wa.w_m;
  ka.w_sh = wa.w_sh;
  ka.stack_check = plan.stack_check ? 1u : 0u;
  ReduceArgs ra;
  ra.acc = ctx->d_acc;
  ra.order = ctx->d_order;
  ra.rgb = rgb_dev;
  ra.sums = sums_dev;
  ra.npix_slots = nps;
  ra.spp = spp;
  ra.pad0 = ra.pad1 = 0;
  // Cross-call pipelining: the launches are numbered across calls (ctx->g_next) and a launch's
  // ring slots (start records, colours, slot counter), scratch parity and render stream follow its
  // global number, so a call whose rings have the previous call's geometry needs no barrier
  // behind it: its warm-up c (c < ring) waits only for the previous call's render that last read
  // that start-record buffer, its render c only for the reduce that last read that colour
  // buffer, and only its last reduce, which writes the caller's image, waits for the caller's
  // stream (ev0).  Back-to-back calls then overlap like the launches inside a call: the next
  // call's first warm-up and renders take the CUs the last launch's draining blocks free.
  // YKGPU_OVERLAP=0 (A/B) keeps every call behind the caller's stream, as do xor128 calls (no
  // warm-up kernel to clear their slot counters) and any call after a failed one.
  const uint64_t g0 = ctx->g_next;
  // (every field that places a launch's start records, colours or per-lane scratch: a call whose
  // K, record size or lane count differs would address other offsets of the same buffers, and its
  // ring waits would not cover the previous call's launches there)
  ykgpu_context::RingGeom geom;
  geom.nps = nps;
  geom.K = K;
  geom.welem = welem;
  geom.warm_ring = kWarmRing;
  geom.col_ring = kColRing;
  geom.lanes = (uint64_t)grid * block;
  geom.id_stride = ctx->id_stride;
  geom.warm = ctx->d_warm;
  geom.col = ctx->d_col;
  geom.mt = ctx->d_mt;
  geom.ids = ctx->d_ids;
  const char* ove = std::getenv("YKGPU_OVERLAP");
  // (the last max(ring) launches, of however many calls, had this geometry: each buffer this call
  // reuses was last used by one of them, whose events ctx->gev holds)
  const bool same_run = ctx->prev_ok && ctx->prev_geom == geom;  // (ctx->run_len continues)
  const bool ov = !x128 && !warm_first && !(ove && std::atoi(ove) == 0) && ctx->prev_ok && ctx->prev_geom == geom &&
                  ctx->run_len >= std::max(kWarmRing, kColRing) && std::max(kWarmRing, kColRing) < kDepRing;
  if (ctx->dirty && (rc = quiesce(ctx))) return rc;  // a failed call's work: wait it out on the host
  const bool after_prev = ctx->prev_enqueued && !ctx->dirty && !ov;
  ctx->prev_ok = false;  // (until this call has been enqueued)
  ctx->dirty = true;
  // slot counters: one per launch of the call for xor128 (cleared here), one per start-record
  // buffer for mt19937 (cleared by the launch's warm-up kernel: a clear between launches as a
  // fill kernel of its own would wait for a free CU behind the warm-ups and reduces, up to 1.6 ms
  // per launch, measured)
  if (std::max(nlaunch, kWarmRing) > ctx->counter_cap) {
    if ((rc = quiesce(ctx))) return rc;
    (void)hipFree(ctx->d_counter);
    (void)hipFree(ctx->d_clk);
    ctx->d_counter = nullptr;
    ctx->d_clk = nullptr;
    ctx->counter_cap = 0;
    YK_HIP(hipMalloc(&ctx->d_counter, std::max(nlaunch, kWarmRing) * sizeof(uint32_t)));
    YK_HIP(hipMalloc(&ctx->d_clk, 4ull * std::max(nlaunch, kWarmRing) * sizeof(unsigned long long)));
    ctx->counter_cap = std::max(nlaunch, kWarmRing);
  }
  // per launch: [0] warm-up start, [1] warm-up end (aux), [2] render start, [3] render end (st),
  // [4] reduce start, [5] reduce end (red); the previous call's stay in lev_prev
  std::swap(ctx->lev, ctx->lev_prev);
  ctx->lev_prev_used = ctx->lev_used;
  while (ctx->lev.size() < 6ull * nlaunch) {
    hipEvent_t e;
    YK_HIP(hipEventCreate(&e));
    ctx->lev.push_back(e);
  }
  ctx->lev_used = 6 * nlaunch;
  // the caller's stream clears this call's slot counters (xor128) and work counters below: before
  // that it waits for the previous call, whose renders may still use both (it may have been
  // enqueued on another stream)
  if (after_prev) YK_HIP(hipStreamWaitEvent(st, ctx->lev_prev[6 * (ctx->prev_n - 1) + 5], 0));
  if (x128) YK_HIP(hipMemsetAsync(ctx->d_counter, 0, nlaunch * sizeof(uint32_t), st));
  if (!ov) {
    YK_HIP(hipMemsetAsync(ctx->d_stats, 0, kCounters * sizeof(unsigned long long), st));
    YK_HIP(hipMemsetAsync(ctx->d_stats + 16, 0xff, 2 * sizeof(unsigned long long), st));  // minima
  }
  YK_HIP(hipEventRecord(ctx->ev0, st));
  if (ov) {
    // (the previous call's last renders may still add their MT-fallback counts here)
    YK_HIP(hipMemsetAsync(ctx->d_stats, 0, kCounters * sizeof(unsigned long long), ctx->aux));
    YK_HIP(hipMemsetAsync(ctx->d_stats + 16, 0xff, 2 * sizeof(unsigned long long), ctx->aux));
  } else {
    // the caller's earlier work, and the whole previous call (its last reduce ends after every
    // launch of it: whichever stream the caller used then), come first
    for (hipStream_t s : {ctx->aux, ctx->red, ctx->alt, ctx->ren}) {
      YK_HIP(hipStreamWaitEvent(s, ctx->ev0, 0));
      if (after_prev) YK_HIP(hipStreamWaitEvent(s, ctx->lev_prev[6 * (ctx->prev_n - 1) + 5], 0));
    }
  }
  while (ctx->gev.size() < 2ull * kDepRing) {
    hipEvent_t e;
    YK_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    ctx->gev.push_back(e);
  }
  // the end of global launch g's render ([0]) or reduce ([1])
  auto gdep = [&](uint64_t g, int which) { return ctx->gev[2 * (g % kDepRing) + which]; };
  auto warm = [&](uint32_t c) -> int {
    hipEvent_t* ev = &ctx->lev[6 * c];
    // its buffer: the render that last read it (launch c - ring, possibly an earlier call's)
    if (c >= kWarmRing)
      YK_HIP(hipStreamWaitEvent(ctx->aux, ctx->lev[6 * (c - kWarmRing) + 3], 0));
    else if (ov)
      YK_HIP(hipStreamWaitEvent(ctx->aux, gdep(g0 + c - kWarmRing, 0), 0));
    wa.s0 = sched[c].first;
    wa.n = (uint64_t)nps * sched[c].second;
    wa.out = ctx->d_warm + (size_t)((g0 + c) % kWarmRing) * nps * K * welem;
    wa.counter = ctx->d_counter + (g0 + c) % kWarmRing;
    const bool defer = !x128 && !f32 && wa.lens && wa.retry_cap && wave_slots(wa.n) <= kDeferSlots;
    const uint32_t wblocks = warm_blocks_for(wa.n, (uint64_t)ctx->cus * warm_per_cu(f32), defer ? kWalkIlp : kWalkIlpInline);
    YK_HIP(hipEventRecord(ev[0], ctx->aux));
    if (!x128) {
      if (f32 && wa.lens)
        hipLaunchKernelGGL((yk_mt_warmup<true, true>), dim3(wblocks), dim3(256), 0, ctx->aux, wa);
      else if (f32)
        hipLaunchKernelGGL((yk_mt_warmup<false, true>), dim3(wblocks), dim3(256), 0, ctx->aux, wa);
      else if (defer)
        hipLaunchKernelGGL(yk_mt_warmup_defer, dim3(wblocks), dim3(256), 0, ctx->aux, wa);
      else if (wa.lens)
        hipLaunchKernelGGL((yk_mt_warmup<true, false>), dim3(wblocks), dim3(256), 0, ctx->aux, wa);
      else
        hipLaunchKernelGGL((yk_mt_warmup<false, false>), dim3(wblocks), dim3(256), 0, ctx->aux, wa);
      YK_HIP(hipGetLastError());
    }
    YK_HIP(hipEventRecord(ev[1], ctx->aux));
    return YK_OK;
  };
  for (uint32_t c = 0; c < std::min(kWarmRing, nlaunch); ++c)
    if ((rc = warm(c))) return rc;
  if (warm_first) YK_HIP(hipStreamSynchronize(ctx->aux));
  uint32_t launches = 0;
  for (uint32_t c = 0; c < nlaunch; ++c) {
    hipEvent_t* ev = &ctx->lev[6 * c];
    const uint32_t s0 = sched[c].first, ks = sched[c].second;
    const uint32_t nsl = nps * ks;
    const uint64_t g = g0 + c;  // the launch's global number (ring slots, parity, stream)
    char* const wring = x128 ? nullptr : ctx->d_warm + (size_t)(g % kWarmRing) * nps * K * welem;
    double* col = ctx->d_col + (size_t)(g % kColRing) * nps * K * kColStride;
    ka.s0 = s0;
    ka.nsl = nsl;
    ka.col = col;
    ka.start = (const void*)wring;
    // Render launches alternate between the caller's stream and ctx->alt: launch c + 1 depends
    // only on its own start records and colour buffer, so its blocks take the CUs that launch c's
    // draining blocks free (per-lane scratch, slot counter and colours are per launch parity)
    const hipStream_t rs = (g & 1) ? ctx->alt : ctx->ren;
    const size_t lanes = (size_t)grid * block;
    ka.mt_scratch = ctx->d_mt ? ctx->d_mt + (g & 1) * lanes * ykd::kMtN : nullptr;
    ka.id_scratch = ctx->d_ids + (g & 1) * lanes * ctx->id_stride;
    YK_HIP(hipStreamWaitEvent(rs, ev[1], 0));  // its start records
    // its colour buffer: the reduce that last read it
    if (c >= kColRing)
      YK_HIP(hipStreamWaitEvent(rs, ctx->lev[6 * (c - kColRing) + 5], 0));
    else if (ov)
      YK_HIP(hipStreamWaitEvent(rs, gdep(g0 + c - kColRing, 1), 0));
    ka.pixel_counter = ctx->d_counter + (x128 ? c : (uint32_t)(g % kWarmRing));
    ka.clk = ctx->d_clk + 4 * c;
#ifdef YK_DRAIN_DIAG
    ka.diag_c = c;
    ka.diag_pad = 0;
#endif
    YK_HIP(hipEventRecord(ev[2], rs));
    const bool count = (ka.flags & YK_FLAG_COUNT_WORK) != 0;
    if (f32)
      hipLaunchKernelGGL(f32_kernel(plan.in_lds, (count ? 1 : 0) | (x128 ? 4 : 0)), dim3(grid), dim3(block),
                         plan.lds_bytes, rs, ka);
    else
      hipLaunchKernelGGL(fp64_kernel(plan.in_lds, (count ? 1 : 0) | (ka.seed_mode == YK_SEED_RANDOM_DEVICE ? 2 : 0) |
                                                      (x128 ? 4 : 0)),
                         dim3(grid), dim3(block), plan.lds_bytes, rs, ka);
    YK_HIP(hipGetLastError());
    YK_HIP(hipEventRecord(ev[3], rs));
    YK_HIP(hipEventRecord(gdep(g, 0), rs));
    ra.col = col;
    ra.nsl = nsl;
    ra.ks = ks;
    ra.first = s0 == 0;
    ra.last = s0 + ks == spp;
    YK_HIP(hipStreamWaitEvent(ctx->red, ev[3], 0));
    if (ov && ra.last) YK_HIP(hipStreamWaitEvent(ctx->red, ctx->ev0, 0));  // the caller's image
    YK_HIP(hipEventRecord(ev[4], ctx->red));
    hipLaunchKernelGGL(yk_reduce_samples, dim3(reduce_blocks(ctx, nps)), dim3(256), 0, ctx->red, ra);
    YK_HIP(hipGetLastError());
    YK_HIP(hipEventRecord(ev[5], ctx->red));
    YK_HIP(hipEventRecord(gdep(g, 1), ctx->red));
    if (c + kWarmRing < nlaunch && (rc = warm(c + kWarmRing))) return rc;
    ++launches;
  }
  YK_HIP(hipStreamWaitEvent(st, ctx->lev[6 * (nlaunch - 1) + 5], 0));  // the caller sees the image
  YK_HIP(hipEventRecord(ctx->ev1, st));
  ctx->g_next = g0 + nlaunch;
  ctx->prev_n = nlaunch;
  ctx->run_len = (same_run ? ctx->run_len : 0) + nlaunch;
  ctx->prev_geom = geom;
  ctx->prev_shape = shape;
  ctx->prev_ok = !x128 && !warm_first;
  ctx->prev_enqueued = true;
  ctx->dirty = false;
  ctx->stats = yk_render_stats{};
  ctx->stats.samples = (uint64_t)p->row_count * tile_width(p) * p->samples_per_pixel;
  ctx->stats.launches = launches;
  ctx->stats.grid_blocks = (uint32_t)grid;
  ctx->stats.launch_spp = K;
  ctx->stats.mem_shrinks = mem_shrinks;
  ctx->stats.seed_key = seed_key;
  // what this call needed (device_bytes: what the context holds)
  {
    const uint64_t lanes = (uint64_t)grid * block;
    uint64_t cb = ctx->t64.bytes + ctx->t32.bytes +
                  (uint64_t)ctx->nspheres * (sizeof(SphereGeo) + sizeof(SphereMat) + sizeof(float4));
    cb += (uint64_t)kColRing * nps * K * kColStride * sizeof(double) + (x128 ? 0 : (uint64_t)kWarmRing * nps * K * welem);
    cb += (nlaunch > 1 ? (uint64_t)nps * 3 * sizeof(double) : 0) + (uint64_t)nps * sizeof(uint32_t);
    cb += nlaunch * sizeof(uint32_t) + kCounters * sizeof(unsigned long long);
    if (retry_cap) cb += retry_n * sizeof(uint4);
    if (!x128) cb += 2 * lanes * ykd::kMtN * sizeof(uint32_t);
    cb += 2 * lanes * std::max(1u, p->max_depth > kStackRegs ? p->max_depth : 1u) * sizeof(uint16_t);
    const uint64_t npix = (uint64_t)p->row_count * tile_width(p);
    cb += npix * 3 + (sums_dev ? npix * 3 * sizeof(double) : 0);
    ctx->stats.call_bytes = cb;
  }
  ctx->stats_pending = true;
  return YK_OK;
}

// Device memory the context holds (yk_render_stats.device_bytes)
uint64_t device_bytes(const ykgpu_context* ctx) {
  uint64_t b = ctx->t64.bytes + ctx->t32.bytes;
  if (ctx->d_geo) b += (uint64_t)ctx->nspheres * (sizeof(SphereGeo) + sizeof(SphereMat) + sizeof(float4));
  b += ctx->warm_cap + ctx->col_cap * sizeof(double) + ctx->acc_cap * sizeof(double);
  b += ctx->retry_cap * sizeof(uint4);
  b += (uint64_t)ctx->order_slots * sizeof(uint32_t) + (uint64_t)ctx->counter_cap * sizeof(uint32_t);
  b += kCounters * sizeof(unsigned long long);
  if (ctx->d_mt) b += 2ull * ctx->scratch_lanes * ykd::kMtN * sizeof(uint32_t);
  if (ctx->d_ids) b += 2ull * ctx->id_lanes * ctx->id_stride * sizeof(uint16_t);
  b += ctx->rgb_cap + ctx->sums_cap * sizeof(double);
  return b;
}

int finish_stats(ykgpu_context* ctx) {
  if (!ctx->stats_pending) return YK_OK;
  YK_HIP(hipEventSynchronize(ctx->ev1));
  float ms = 0;
  YK_HIP(hipEventElapsedTime(&ms, ctx->ev0, ctx->ev1));
  unsigned long long c[kCounters];
  YK_HIP(hipMemcpy(c, ctx->d_stats, sizeof(c), hipMemcpyDeviceToHost));
  ctx->stats.node_visits = c[4];
  ctx->stats.linear_scans = c[5];
  ctx->stats.newton_calls = c[6];
  ctx->stats.newton_iters = c[7];
  for (int k = 0; k < 8; ++k) ctx->stats.phase_cycles[k] = c[8 + k];
  for (int k = 0; k < 3; ++k) ctx->stats.timeline[k] = c[16 + k];
  for (int k = 0; k < 4; ++k) ctx->stats.diag[k] = c[19 + k];
  for (int k = 0; k < 8; ++k) ctx->stats.work[k] = c[24 + k];
  ctx->stats.total_ms = ms;
  double tw = 0, tr = 0, tp = 0, busy = 0;
  for (uint32_t k = 0; k + 5 < ctx->lev_used; k += 6) {
    float a = 0, b = 0, c = 0;
    YK_HIP(hipEventSynchronize(ctx->lev[k + 5]));
    YK_HIP(hipEventElapsedTime(&a, ctx->lev[k], ctx->lev[k + 1]));
    YK_HIP(hipEventElapsedTime(&b, ctx->lev[k + 2], ctx->lev[k + 3]));
    YK_HIP(hipEventElapsedTime(&c, ctx->lev[k + 4], ctx->lev[k + 5]));
    tw += a, tr += b, tp += c;
    // union of the render spans: launch k/6 overlaps only the tail of the one before it
    float ov = 0;
    if (k >= 6) YK_HIP(hipEventElapsedTime(&ov, ctx->lev[k + 2], ctx->lev[k - 6 + 3]));
    busy += b - std::min<double>(b, std::max<double>(0.0, ov));
  }
  ctx->stats.render_busy_ms = busy;
  // the shader clock of each launch (YK_CLOCK_* probe: wave 0 of block 0), averaged over the call
  // weighted by the probe's real time
  const uint32_t nl = ctx->lev_used / 6;
  std::vector<unsigned long long> clk(4ull * nl);
  std::vector<double> mhz(nl, 0.0);
  if (nl) YK_HIP(hipMemcpy(clk.data(), ctx->d_clk, clk.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  double cyc = 0, real = 0;
  for (uint32_t k = 0; k < nl; ++k) {
    const double dc = (double)(clk[4 * k + 2] - clk[4 * k]), dr = (double)(clk[4 * k + 3] - clk[4 * k + 1]);
    if (dr > 0 && clk[4 * k + 3] > clk[4 * k + 1]) {
      mhz[k] = dc / dr * 100.0;  // s_memrealtime ticks at 100 MHz
      cyc += dc;
      real += dr;
    }
  }
  ctx->stats.sclk_mhz = real > 0 ? cyc / real * 100.0 : 0.0;
  if (std::getenv("YKGPU_TIMELINE")) {  // diagnostic: per-launch event times (ms from the call's start)
    // the previous call's launches on the same clock (negative: before this call's start), so the
    // handover between back-to-back calls shows
    for (uint32_t k = 0; k + 5 < ctx->lev_prev_used && k + 5 < ctx->lev_prev.size(); k += 6) {
      float t[6];
      bool ok = true;
      for (int q = 0; q < 6 && ok; ++q) ok = hipEventElapsedTime(&t[q], ctx->ev0, ctx->lev_prev[k + q]) == hipSuccess;
      if (!ok) {
        (void)hipGetLastError();
        break;
      }
      std::fprintf(stderr, "prev   %u: warm %8.3f %8.3f  render %8.3f %8.3f  reduce %8.3f %8.3f\n", k / 6, t[0],
                   t[1], t[2], t[3], t[4], t[5]);
    }
    for (uint32_t k = 0; k + 5 < ctx->lev_used; k += 6) {
      float t[6];
      for (int q = 0; q < 6; ++q) YK_HIP(hipEventElapsedTime(&t[q], ctx->ev0, ctx->lev[k + q]));
      std::fprintf(stderr, "launch %u: warm %8.3f %8.3f  render %8.3f %8.3f  reduce %8.3f %8.3f  sclk %7.1f MHz\n",
                   k / 6, t[0], t[1], t[2], t[3], t[4], t[5], mhz[k / 6]);
    }
    std::fprintf(stderr, "call %8.3f\n", ms);
  }
  ctx->stats.warmup_ms = tw;
  ctx->stats.kernel_ms = tr;
  ctx->stats.resolve_ms = tp;
  ctx->stats.segments = c[0];
  ctx->stats.sphere_tests = c[1];
  ctx->stats.sqrt_calls = c[2];
  ctx->stats.mt_fallbacks = c[3];
  ctx->stats.device_bytes = device_bytes(ctx);
  ctx->stats_pending = false;
  return YK_OK;
}

// Builds one BVH over the scene and uploads it into t: `geo` holds the tuple-order geometry the
// kernel's leaves read (`elem` bytes per sphere), stored in leaf order; kern[v][lds] are the kernel
// instances of workgroup size v (kBlock, kBlockX128) that read the tree from global memory / LDS
// (for the occupancy).
int upload_tree(ykgpu_context* ctx, DevTree& t, const std::vector<double>& centers, const std::vector<double>& radii,
                double cam_ext, const ykbvh::Options& opt, uint32_t leaf_cap, const void* geo, size_t elem,
                size_t tgeo_elem, const RenderKernel (&kern)[2][2], bool exact_stack) {
  const uint32_t count = (uint32_t)radii.size();
  if (opt.max_leaf > leaf_cap) return fail(YK_ERR_UNSUPPORTED, "BVH leaf size above the kernel's leaf capacity");
  const ykbvh::Built bvh = ykbvh::build(centers.data(), radii.data(), count, cam_ext, opt);
  if (bvh.depth > ykbvh::kMaxDepth) return fail(YK_ERR_INVALID, "BVH deeper than the traversal stack");
  std::vector<char> leaf_geo(count * elem);
  for (uint32_t i = 0; i < count; ++i)
    std::memcpy(leaf_geo.data() + i * elem, (const char*)geo + (size_t)bvh.order[i] * elem, elem);
  t.release();
  int32_t root_code = 0;
  uint32_t wdepth = 0;
  const std::vector<DevNode> snodes = ykbvh::wide_nodes(bvh, &root_code, &wdepth);
  // every leaf the kernel can reach must fit its leaf code (kLeafCapF64 / kLeafCapF32)
  auto leaf_fits = [&](int32_t code) { return code >= 0 || (((~(uint32_t)code) & 15u) <= leaf_cap); };
  bool fits = leaf_fits(root_code);
  for (const DevNode& w : snodes)
    for (int k = 0; k < 4; ++k) fits = fits && leaf_fits(w.child[k]);
  if (!fits) return fail(YK_ERR_UNSUPPORTED, "a BVH leaf holds more spheres than the kernel's leaf code tests");
  const size_t nn = std::max<size_t>(1, snodes.size());
  YK_HIP(hipMalloc(&t.nodes, nn * sizeof(DevNode)));
  YK_HIP(hipMalloc(&t.leaf_geo, count * elem));
  YK_HIP(hipMalloc(&t.leaf_ids, count * sizeof(uint32_t)));
  if (!snodes.empty())
    YK_HIP(hipMemcpy(t.nodes, snodes.data(), snodes.size() * sizeof(DevNode), hipMemcpyHostToDevice));
  YK_HIP(hipMemcpy(t.leaf_geo, leaf_geo.data(), count * elem, hipMemcpyHostToDevice));
  YK_HIP(hipMemcpy(t.leaf_ids, bvh.order.data(), count * sizeof(uint32_t), hipMemcpyHostToDevice));
  t.bytes = nn * sizeof(DevNode) + count * elem + count * sizeof(uint32_t);
  t.root = root_code;
  t.depth = bvh.depth;
  t.origin_bound = bvh.origin_bound;
  t.n_nodes = (uint32_t)snodes.size();
  // LDS layout: [nodes][leaf geometry][leaf ids][tuple-order geometry][materials][traversal
  // stacks].  The tables (tgeo_elem bytes of tuple-order geometry per sphere — the FP64 kernel's
  // SphereGeo, the FP32 kernel's float4 — and the SphereMat: candidate roots, shading, unwind) go
  // wherever the tree goes: the LDS instance reads both from LDS.  One
  // plan per workgroup size (the stacks are per lane).
  auto a16 = [](size_t b) { return (b + 15) & ~size_t(15); };
  const size_t scene_bytes = a16(t.n_nodes * sizeof(DevNode)) + a16(count * elem) + a16(count * sizeof(uint32_t));
  const size_t tgeo_bytes = tgeo_elem ? a16(count * tgeo_elem) : 0;
  const size_t mat_bytes = tgeo_elem ? a16(count * sizeof(SphereMat)) : 0;
  t.geo_off = (uint32_t)a16(t.n_nodes * sizeof(DevNode));
  t.ids_off = t.geo_off + (uint32_t)a16(count * elem);
  for (int v = 0; v < 2; ++v) {
    DevTree::Plan& pl = t.plan[v];
    // threads per workgroup = traversal stacks per workgroup
    const int blk = block_of(v == 1);
    const int rays = blk;
    // a CU holds one workgroup of >= 512 threads (768 / blk of smaller ones); 2 KB below the
    // share: the hardware's allocation granularity (3 blocks of 54144 bytes measured only 2
    // resident per CU)
    const size_t budget = (size_t)160 * 1024 / (blk >= 512 ? 1 : 768 / blk) - 2048;
    const size_t min_stacks = (size_t)12 * rays * 4;
    pl.in_lds = scene_bytes + tgeo_bytes + mat_bytes + min_stacks <= budget;
    const size_t tables = pl.in_lds ? tgeo_bytes + mat_bytes : 0;
    // Traversal stack per lane: up to 3 pushes per wide level suffice (3 * wdepth + 1 entries);
    // the capacity is what still fits the budget (at least 8); a lane that would exceed it
    // abandons the traversal for the exact linear scan.  Pushes write unconditionally at the
    // current top (up to 3 past the capacity): +4 entries.
    {
      const size_t used = pl.in_lds ? scene_bytes + tables : 0;
      const uint32_t fit = used + min_stacks <= budget ? (uint32_t)((budget - used) / (rays * 4)) : 12u;
      pl.stack_cap = std::max(8u, std::min(3 * wdepth + 1, fit - 4));
      pl.stack_entries = pl.stack_cap + 4;
      pl.stack_check = true;
      // The FP64 branch-free visit (exact_stack) with 3 * wdepth + 1 entries: a visit at inner
      // level k finds at most 3 entries per ancestor level on the stack (depth-first: what is left
      // of an ancestor's up to 3 pushes; the sentinel is entry 0), so its top is <= 3k + 1 <=
      // 3 * wdepth - 2, its writes (at the top and the next two entries) stay below entry
      // 3 * wdepth and its new top is <= 3 * wdepth + 1: no overflow, no check, no slack
      if (exact_stack && fit >= 3 * wdepth + 1) {
        pl.stack_cap = 3 * wdepth + 1;
        pl.stack_entries = pl.stack_cap;
        pl.stack_check = false;
      }
#ifdef YK_STACK_CAP_FORCE
      // (test builds, tests/test_gpu_robust.py: a checked stack this shallow overflows, and the
      // lanes that overflow take the exact linear scan)
      pl.stack_cap = YK_STACK_CAP_FORCE;
      pl.stack_entries = pl.stack_cap + 4;
      pl.stack_check = true;
#endif
    }
    pl.tgeo_off = pl.in_lds && tgeo_elem ? (uint32_t)scene_bytes : 0u;
    pl.mat_off = pl.in_lds && tgeo_elem ? (uint32_t)(scene_bytes + tgeo_bytes) : 0u;
    pl.stack_off = pl.in_lds ? (uint32_t)(scene_bytes + tables) : 0u;
    pl.lds_bytes = pl.stack_off + pl.stack_entries * rays * (uint32_t)sizeof(int32_t);
    int per_cu = 0;
    const RenderKernel k = kern[v][pl.in_lds ? 1 : 0];
    const hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, blk, pl.lds_bytes);
    if (e != hipSuccess || per_cu < 1) per_cu = 1;
    pl.grid = per_cu * ctx->cus;
  }
  return YK_OK;
}

}  // namespace

extern "C" {

uint32_t ykgpu_abi_version(void) { return YKGPU_ABI_VERSION; }

#ifdef YK_DRAIN_DIAG
// (diagnostic builds only, tools/drain_probe.py) the wave records since the last clear:
// [launch][block][wave] x {start, end, HW_ID | XCC_ID << 32}
int ykgpu_diag_wave_times(unsigned long long* out, size_t n) {
  const size_t cap = sizeof(yk_wave_times) / sizeof(unsigned long long);
  YK_HIP(hipDeviceSynchronize());
  YK_HIP(hipMemcpyFromSymbol(out, HIP_SYMBOL(yk_wave_times), std::min(n, cap) * sizeof(unsigned long long)));
  return YK_OK;
}
int ykgpu_diag_wave_times_clear(void) {
  YK_HIP(hipDeviceSynchronize());
  static std::vector<unsigned long long> z(sizeof(yk_wave_times) / sizeof(unsigned long long), 0ull);
  YK_HIP(hipMemcpyToSymbol(HIP_SYMBOL(yk_wave_times), z.data(), z.size() * sizeof(unsigned long long)));
  return YK_OK;
}
#endif

const char* ykgpu_last_error(void) { return g_last_error.c_str(); }

int ykgpu_device_count(int* count) {
  if (!count) return fail(YK_ERR_INVALID, "null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return fail(YK_ERR_DEVICE, std::string("hipGetDeviceCount: ") + hipGetErrorString(e));
  }
  *count = n;
  return YK_OK;
}

int ykgpu_context_create(int device, ykgpu_context** out) {
  if (!out) return fail(YK_ERR_INVALID, "null out");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
    return fail(YK_ERR_DEVICE, "no HIP device (the renderer has no CPU fallback)");
  if (device < 0 || device >= n) return fail(YK_ERR_INVALID, "device index out of range");
  YK_HIP(hipSetDevice(device));
  hipDeviceProp_t prop;
  YK_HIP(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(YK_ERR_DEVICE, std::string("built for gfx950, device is ") + prop.gcnArchName);
  auto* ctx = new ykgpu_context();
  ctx->device = device;
  ctx->cus = prop.multiProcessorCount;
  for (int k16 = 0; k16 < 16; ++k16)
    (void)hipFuncSetAttribute((const void*)fp64_kernel(k16 & 8, k16 & 7), hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
  for (int k8 = 0; k8 < 8; ++k8)
    (void)hipFuncSetAttribute((const void*)f32_kernel(k8 & 4, (k8 & 1) | ((k8 & 2) << 1)),
                              hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  if (hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking) != hipSuccess ||
#if YK_RED_PRIO
      create_render_stream(&ctx->red) != hipSuccess ||  // (A/B: the reduces at the renders' priority)
#else
      hipStreamCreateWithFlags(&ctx->red, hipStreamNonBlocking) != hipSuccess ||
#endif
      create_render_stream(&ctx->alt) != hipSuccess || create_render_stream(&ctx->ren) != hipSuccess ||
      hipEventCreate(&ctx->ev0) != hipSuccess || hipEventCreate(&ctx->ev1) != hipSuccess ||
      hipMalloc(&ctx->d_stats, kCounters * sizeof(unsigned long long)) != hipSuccess) {
    ykgpu_context_destroy(ctx);
    return fail(YK_ERR_DEVICE, "context resources");
  }
  *out = ctx;
  return YK_OK;
}

int ykgpu_context_destroy(ykgpu_context* ctx) {
  if (!ctx) return YK_OK;
  (void)hipSetDevice(ctx->device);
  if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
  (void)hipFree(ctx->d_geo);
  (void)hipFree(ctx->d_mat);
  (void)hipFree(ctx->d_geo_f);
  (void)hipFree(ctx->d_counter);
  (void)hipFree(ctx->d_clk);
  (void)hipFree(ctx->d_stats);
  (void)hipFree(ctx->d_warm);
  (void)hipFree(ctx->d_retry);
  (void)hipFree(ctx->d_order);
  (void)hipFree(ctx->d_col);
  (void)hipFree(ctx->d_acc);
  ctx->t64.release();
  ctx->t32.release();
  (void)hipFree(ctx->d_mt);
  (void)hipFree(ctx->d_ids);
  (void)hipFree(ctx->d_rgb);
  (void)hipFree(ctx->d_sums);
  for (hipEvent_t e : ctx->lev) (void)hipEventDestroy(e);
  for (hipEvent_t e : ctx->lev_prev) (void)hipEventDestroy(e);
  for (hipEvent_t e : ctx->gev) (void)hipEventDestroy(e);
  if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
  if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
  if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
  if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
  if (ctx->red) (void)hipStreamDestroy(ctx->red);
  if (ctx->alt) (void)hipStreamDestroy(ctx->alt);
  if (ctx->ren) (void)hipStreamDestroy(ctx->ren);
  delete ctx;
  return YK_OK;
}

int ykgpu_set_scene(ykgpu_context* ctx, const yk_sphere* spheres, uint32_t count,
                    const yk_camera* camera) {
  if (!ctx || !spheres || !camera) return fail(YK_ERR_INVALID, "null argument");
  if (count == 0 || count > 65535) return fail(YK_ERR_INVALID, "sphere count must be 1..65535");
  std::vector<SphereGeo> geo(count);
  std::vector<SphereMat> mat(count);
  std::vector<float4> geo_f(count);
  for (uint32_t i = 0; i < count; ++i) {
    const yk_sphere& s = spheres[i];
    if (s.material > YK_MATERIAL_DIELECTRIC) return fail(YK_ERR_INVALID, "unknown material kind");
    geo[i] = {s.center[0], s.center[1], s.center[2], s.radius * s.radius};
    // sphere<float>: centre and radius rounded to float, radius*radius a float product
    const float rf = (float)s.radius;
    geo_f[i] = make_float4((float)s.center[0], (float)s.center[1], (float)s.center[2], rf * rf);
    mat[i] = {s.albedo[0], s.albedo[1], s.albedo[2], s.fuzz, s.radius, s.ior, s.material, 0.0f, 0.0};  // inv_r*: yk_mat_prep
#if YK_DIEL_PRE
    if (s.material == YK_MATERIAL_DIELECTRIC) {
      // the FP64 kernel's dielectric reads 1/ior and Schlick's r0 for both sides of the surface
      // from its otherwise unused fields (never unwound: its attenuation is 1), computed here
      // with the operations and order of ykd::reflectance (IEEE double, no contraction)
      const double inv = 1.0 / s.ior;
      double r0f = (1 - inv) / (1 + inv), r0b = (1 - s.ior) / (1 + s.ior);
      r0f = r0f * r0f;
      r0b = r0b * r0b;
      mat[i].fuzz = inv;
      mat[i].ar = r0f;
      mat[i].ag = r0b;
    }
#endif
  }
  YK_HIP(hipSetDevice(ctx->device));
  // a render enqueued by ykgpu_render_async on the caller's stream (and its launches on the
  // context's own streams) may still read the scene: wait for this context's last call — ev1
  // follows the call's final reduce, which follows every launch of the call (launch()) — and for
  // its own stream (the diagnostic entry points), not for the rest of the device
  YK_HIP(hipEventSynchronize(ctx->ev1));
  YK_HIP(hipStreamSynchronize(ctx->stream));
  // ... and for every stream of the context: a launch() that failed part-way may have queued
  // warm-ups, renders or reduces without recording ev1 (still not the rest of the device)
  for (hipStream_t s : {ctx->aux, ctx->red, ctx->ren, ctx->alt}) YK_HIP(hipStreamSynchronize(s));
  if (count > ctx->nspheres || !ctx->d_geo) {
    (void)hipFree(ctx->d_geo);
    (void)hipFree(ctx->d_mat);
    (void)hipFree(ctx->d_geo_f);
    ctx->d_geo = nullptr;
    ctx->d_mat = nullptr;
    ctx->d_geo_f = nullptr;
    YK_HIP(hipMalloc(&ctx->d_geo, count * sizeof(SphereGeo)));
    YK_HIP(hipMalloc(&ctx->d_mat, count * sizeof(SphereMat)));
    YK_HIP(hipMalloc(&ctx->d_geo_f, count * sizeof(float4)));
  }
  YK_HIP(hipMemcpy(ctx->d_geo, geo.data(), count * sizeof(SphereGeo), hipMemcpyHostToDevice));
  YK_HIP(hipMemcpy(ctx->d_geo_f, geo_f.data(), count * sizeof(float4), hipMemcpyHostToDevice));
  // the BVHs (culling only): the FP64 kernel's and the FP32 kernel's, whose boxes
  // also carry render<float>'s sphere-test error (§4.1)
  std::vector<double> centers(3 * size_t(count)), radii(count);
  double rmin = INFINITY;
  for (uint32_t i = 0; i < count; ++i) {
    for (int k = 0; k < 3; ++k) centers[3 * i + k] = spheres[i].center[k];
    radii[i] = spheres[i].radius;
    rmin = std::min(rmin, std::fabs(radii[i]));
  }
  double cam_ext = 0;
  for (int k = 0; k < 3; ++k) cam_ext = std::max(cam_ext, std::fabs(camera->origin[k]));
  // one sphere per leaf for the 4-wide FP64 tree: 64-spp A/B on the final scene 32.5 -> 31.7 ms
  // against two (three: 33.4); the FP32 tree keeps two (one or three: neutral)
  ykbvh::Options bopt;
  bopt.max_leaf = kLeafCapF64;  // the FP64 kernel tests one sphere per leaf, without a loop
  if (const char* e = ab_knob("YKGPU_BVH_BINS")) bopt.bins = std::max(2, std::min(256, std::atoi(e)));  // (A/B)
  // SAH over all three axes: 512-spp A/B 199.4 -> 198.3 ms (model: 5.51 -> 5.13 visits per segment)
  bopt.all_axes = true;
  if (const char* e = ab_knob("YKGPU_BVH_ALLAXES")) bopt.all_axes = std::atoi(e) != 0;                  // (A/B)
  const RenderKernel k64[2][2] = {{fp64_kernel(false, 0), fp64_kernel(true, 0)},
                                  {fp64_kernel(false, 4), fp64_kernel(true, 4)}};
  int rc = upload_tree(ctx, ctx->t64, centers, radii, cam_ext, bopt, kLeafCapF64, geo.data(), sizeof(SphereGeo),
                       sizeof(SphereGeo), k64, YK_NODE_BF != 0 && YK_STACK_EXACT != 0);
  if (rc) return rc;
  ykbvh::Options fopt = bopt;
  fopt.max_leaf = kLeafCapF32;  // the FP32 kernel's leaf loop is unrolled for two spheres
  if (const char* e = ab_knob("YKGPU_BVH_ALLAXES_F32")) fopt.all_axes = std::atoi(e) != 0;  // (A/B; on: neutral)
  fopt.radius_grow = 2.0 * (double)ykbvh::kF32Cone;
  fopt.f32_big = ab_knob("YKGPU_F32_NO_BIG") == nullptr;  // (A/B: the cone bound alone)
  const RenderKernel k32[2][2] = {{f32_kernel(false, 0), f32_kernel(true, 0)},
                                  {f32_kernel(false, 4), f32_kernel(true, 4)}};
  rc = upload_tree(ctx, ctx->t32, centers, radii, cam_ext, fopt, kLeafCapF32, geo_f.data(), sizeof(float4),
                   sizeof(float4), k32, false);
  if (rc) return rc;
  // the float bound assumes neither underflow nor overflow: a scene outside that
  // scale renders FP32 with the linear scan throughout
  if (!(rmin >= 0x1p-20) || !(ctx->t32.origin_bound <= 0x1p20)) ctx->t32.origin_bound = -1.0;
  YK_HIP(hipMemcpy(ctx->d_mat, mat.data(), count * sizeof(SphereMat), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(yk_mat_prep, dim3((count + 255) / 256), dim3(256), 0, ctx->stream, ctx->d_mat, count);
  YK_HIP(hipGetLastError());
  YK_HIP(hipStreamSynchronize(ctx->stream));
  ctx->nspheres = count;
  ctx->cam = *camera;
  ctx->have_scene = true;
  return YK_OK;
}

int ykgpu_render_async(ykgpu_context* ctx, const yk_render_params* p, void* rgb_device,
                       void* stream) {
  int rc = check_params(ctx, p);
  if (rc) return rc;
  if (!rgb_device) return fail(YK_ERR_INVALID, "null output");
  YK_HIP(hipSetDevice(ctx->device));
  hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
  ctx->t0 = std::chrono::steady_clock::now();
  return launch(ctx, p, (uint8_t*)rgb_device, nullptr, st);
}

static int render_host(ykgpu_context* ctx, const yk_render_params* p, uint8_t* rgb_host,
                       double* sums_host) {
  int rc = check_params(ctx, p);
  if (rc) return rc;
  YK_HIP(hipSetDevice(ctx->device));
  const auto t0 = std::chrono::steady_clock::now();
  const size_t npix = (size_t)p->row_count * tile_width(p);
  if (npix * 3 > ctx->rgb_cap) {
    (void)hipFree(ctx->d_rgb);
    ctx->d_rgb = nullptr;
    YK_HIP(hipMalloc(&ctx->d_rgb, npix * 3));
    ctx->rgb_cap = npix * 3;
  }
  if (sums_host && npix * 3 > ctx->sums_cap) {
    (void)hipFree(ctx->d_sums);
    ctx->d_sums = nullptr;
    YK_HIP(hipMalloc(&ctx->d_sums, npix * 3 * sizeof(double)));
    ctx->sums_cap = npix * 3;
  }
  rc = launch(ctx, p, ctx->d_rgb, sums_host ? ctx->d_sums : nullptr, ctx->stream);
  if (rc) return rc;
  if (rgb_host) YK_HIP(hipMemcpyAsync(rgb_host, ctx->d_rgb, npix * 3, hipMemcpyDeviceToHost, ctx->stream));
  if (sums_host)
    YK_HIP(hipMemcpyAsync(sums_host, ctx->d_sums, npix * 3 * sizeof(double), hipMemcpyDeviceToHost,
                          ctx->stream));
  YK_HIP(hipStreamSynchronize(ctx->stream));
  rc = finish_stats(ctx);
  ctx->stats.total_ms =
      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return rc;
}

int ykgpu_render(ykgpu_context* ctx, const yk_render_params* p, uint8_t* rgb_host) {
  if (!rgb_host) return fail(YK_ERR_INVALID, "null output");
  return render_host(ctx, p, rgb_host, nullptr);
}

int ykgpu_render_trace(ykgpu_context* ctx, const yk_render_params* p, uint32_t max_rays, double* rays_host,
                       uint32_t* counts_host) {
  int rc = check_params(ctx, p);
  if (rc) return rc;
  if (!max_rays || !rays_host || !counts_host) return fail(YK_ERR_INVALID, "null output or max_rays == 0");
  const size_t n = (size_t)p->row_count * tile_width(p) * p->samples_per_pixel;
  YK_HIP(hipSetDevice(ctx->device));
  YK_HIP(hipMalloc(&ctx->d_trace, n * max_rays * 6 * sizeof(double)));
  if (hipMalloc(&ctx->d_trace_counts, n * sizeof(uint32_t)) != hipSuccess) {
    (void)hipFree(ctx->d_trace);
    ctx->d_trace = nullptr;
    return fail(YK_ERR_NOMEM, "ykgpu_render_trace: ray counts");
  }
  ctx->trace_cap = max_rays;
  yk_render_params q = *p;
  q.flags |= YK_FLAG_COUNT_WORK | YK_FLAG_TRACE_RAYS;
  rc = render_host(ctx, &q, nullptr, nullptr);
  hipError_t e = hipSuccess;
  if (!rc) e = hipMemcpy(rays_host, ctx->d_trace, n * max_rays * 6 * sizeof(double), hipMemcpyDeviceToHost);
  if (!rc && e == hipSuccess) e = hipMemcpy(counts_host, ctx->d_trace_counts, n * sizeof(uint32_t), hipMemcpyDeviceToHost);
  (void)hipFree(ctx->d_trace);
  (void)hipFree(ctx->d_trace_counts);
  ctx->d_trace = nullptr;
  ctx->d_trace_counts = nullptr;
  ctx->trace_cap = 0;
  if (rc) return rc;
  if (e != hipSuccess) return fail(YK_ERR_DEVICE, std::string("ykgpu_render_trace: ") + hipGetErrorString(e));
  return YK_OK;
}

int ykgpu_render_sums(ykgpu_context* ctx, const yk_render_params* p, double* sums_host) {
  if (!sums_host) return fail(YK_ERR_INVALID, "null output");
  return render_host(ctx, p, nullptr, sums_host);
}

int ykgpu_math_sqrt(ykgpu_context* ctx, const double* in, double* out, uint64_t n) {
  if (!ctx || (n && (!in || !out))) return fail(YK_ERR_INVALID, "null argument");
  if (n == 0) return YK_OK;
  YK_HIP(hipSetDevice(ctx->device));
  double* d = nullptr;
  YK_HIP(hipMalloc(&d, 2 * n * sizeof(double)));
  hipError_t e = hipMemcpy(d, in, n * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    const uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(yk_math_sqrt, dim3((uint32_t)blocks), dim3(256), 0, ctx->stream, d, d + n, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e == hipSuccess) e = hipMemcpy(out, d + n, n * sizeof(double), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(YK_ERR_DEVICE, std::string("ykgpu_math_sqrt: ") + hipGetErrorString(e));
  return YK_OK;
}

int ykgpu_math_sqrt_f32(ykgpu_context* ctx, const float* in, float* out, uint64_t n) {
  if (!ctx || (n && (!in || !out))) return fail(YK_ERR_INVALID, "null argument");
  if (n == 0) return YK_OK;
  YK_HIP(hipSetDevice(ctx->device));
  float* d = nullptr;
  YK_HIP(hipMalloc(&d, 2 * n * sizeof(float)));
  hipError_t e = hipMemcpy(d, in, n * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    const uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(yk_math_sqrt_f32, dim3((uint32_t)blocks), dim3(256), 0, ctx->stream, d, d + n, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e == hipSuccess) e = hipMemcpy(out, d + n, n * sizeof(float), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(YK_ERR_DEVICE, std::string("ykgpu_math_sqrt_f32: ") + hipGetErrorString(e));
  return YK_OK;
}

int ykgpu_math_div(ykgpu_context* ctx, const double* num3, const double* den, double* out3, uint64_t n) {
  if (!ctx || (n && (!num3 || !den || !out3))) return fail(YK_ERR_INVALID, "null argument");
  if (n == 0) return YK_OK;
  YK_HIP(hipSetDevice(ctx->device));
  double* d = nullptr;
  YK_HIP(hipMalloc(&d, 7 * n * sizeof(double)));
  hipError_t e = hipMemcpy(d, num3, 3 * n * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d + 3 * n, den, n * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    const uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(yk_math_div, dim3((uint32_t)blocks), dim3(256), 0, ctx->stream, d, d + 3 * n, d + 4 * n, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e == hipSuccess) e = hipMemcpy(out3, d + 4 * n, 3 * n * sizeof(double), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(YK_ERR_DEVICE, std::string("ykgpu_math_div: ") + hipGetErrorString(e));
  return YK_OK;
}

int ykgpu_math_div_f32(ykgpu_context* ctx, const float* num3, const float* den, float* out3, uint64_t n) {
  if (!ctx || (n && (!num3 || !den || !out3))) return fail(YK_ERR_INVALID, "null argument");
  if (n == 0) return YK_OK;
  YK_HIP(hipSetDevice(ctx->device));
  float* d = nullptr;
  YK_HIP(hipMalloc(&d, 7 * n * sizeof(float)));
  hipError_t e = hipMemcpy(d, num3, 3 * n * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d + 3 * n, den, n * sizeof(float), hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    const uint64_t blocks = (n + 255) / 256;
    hipLaunchKernelGGL(yk_math_div_f32, dim3((uint32_t)blocks), dim3(256), 0, ctx->stream, d, d + 3 * n, d + 4 * n, n);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  if (e == hipSuccess) e = hipMemcpy(out3, d + 4 * n, 3 * n * sizeof(float), hipMemcpyDeviceToHost);
  (void)hipFree(d);
  if (e != hipSuccess) return fail(YK_ERR_DEVICE, std::string("ykgpu_math_div_f32: ") + hipGetErrorString(e));
  return YK_OK;
}

int ykgpu_get_stats(ykgpu_context* ctx, yk_render_stats* out) {
  if (!ctx || !out) return fail(YK_ERR_INVALID, "null argument");
  YK_HIP(hipSetDevice(ctx->device));
  int rc = finish_stats(ctx);
  if (rc) return rc;
  *out = ctx->stats;
  return YK_OK;
}

// ---- several devices in one process (include/ykgpu.h "several devices") ----------------------
// One context per entry; rows dealt cyclically over the entries (tile row t of the call's row set
// → entry t mod k, uecraytracing_amd/tiles.py's dealing); every entry renders its tile into a
// device buffer on its own streams, and the tile is copied from its device straight into its rows
// of the caller's host image by one strided 2-D copy: the image ends on the host anyway (stb
// writes it), so a device-side gather first would only add a hop.
int ykgpu_group_create(const int* devices, uint32_t n_devices, ykgpu_group** out) {
  if (!out) return fail(YK_ERR_INVALID, "null out");
  *out = nullptr;
  if (!devices || n_devices == 0) return fail(YK_ERR_INVALID, "empty device list");
  if (n_devices > 64) return fail(YK_ERR_INVALID, "at most 64 entries per group");
  auto* g = new ykgpu_group();
  for (uint32_t k = 0; k < n_devices; ++k) {
    ykgpu_context* c = nullptr;
    const int rc = ykgpu_context_create(devices[k], &c);
    if (rc) {
      const std::string msg = g_last_error;
      ykgpu_group_destroy(g);
      return fail(rc, "group entry " + std::to_string(k) + " (device " + std::to_string(devices[k]) + "): " + msg);
    }
    g->ctx.push_back(c);
  }
  g->tile.assign(n_devices, nullptr);
  g->tile_cap.assign(n_devices, 0);
  g->st.assign(n_devices, yk_render_stats{});
  *out = g;
  return YK_OK;
}

int ykgpu_group_destroy(ykgpu_group* g) {
  if (!g) return YK_OK;
  for (size_t k = 0; k < g->ctx.size(); ++k) {
    if (k < g->tile.size() && g->tile[k]) {
      (void)hipSetDevice(g->ctx[k]->device);
      (void)hipStreamSynchronize(g->ctx[k]->stream);
      (void)hipFree(g->tile[k]);
    }
    ykgpu_context_destroy(g->ctx[k]);
  }
  delete g;
  return YK_OK;
}

int ykgpu_group_size(const ykgpu_group* g, uint32_t* n) {
  if (!g || !n) return fail(YK_ERR_INVALID, "null argument");
  *n = (uint32_t)g->ctx.size();
  return YK_OK;
}

int ykgpu_group_set_scene(ykgpu_group* g, const yk_sphere* spheres, uint32_t count, const yk_camera* camera) {
  if (!g) return fail(YK_ERR_INVALID, "null group");
  for (ykgpu_context* c : g->ctx) {
    const int rc = ykgpu_set_scene(c, spheres, count, camera);
    if (rc) return rc;
  }
  return YK_OK;
}

int ykgpu_group_render(ykgpu_group* g, const yk_render_params* p, uint8_t* rgb_host) {
  if (!g || !p || !rgb_host) return fail(YK_ERR_INVALID, "null argument");
  const uint32_t k = (uint32_t)g->ctx.size();
  int rc = check_params(g->ctx[0], p);
  if (rc) return rc;
  if (k > 1 && p->row_band_log2 != 0)
    return fail(YK_ERR_UNSUPPORTED, "a group deals single rows: row_band_log2 must be 0");
  if (k > 1 && (uint64_t)p->row_stride * k >= (1ull << 32)) return fail(YK_ERR_INVALID, "row_stride * devices overflows");
  const auto t0 = std::chrono::steady_clock::now();
  const size_t row_bytes = (size_t)tile_width(p) * 3;
  std::vector<yk_render_params> sub(k, *p);
  std::vector<uint32_t> rows(k, 0);
  // 1. every entry's tile enqueued on its own device before any copy: the devices run together
  for (uint32_t e = 0; e < k; ++e) {
    rows[e] = p->row_count > e ? (p->row_count - e + k - 1) / k : 0;
    if (!rows[e]) continue;
    sub[e].row_begin = p->row_begin + e * p->row_stride;
    sub[e].row_stride = p->row_stride * k;
    sub[e].row_count = rows[e];
    ykgpu_context* c = g->ctx[e];
    YK_HIP(hipSetDevice(c->device));
    const size_t need = rows[e] * row_bytes;
    if (need > g->tile_cap[e]) {
      (void)hipStreamSynchronize(c->stream);
      (void)hipFree(g->tile[e]);
      g->tile[e] = nullptr;
      g->tile_cap[e] = 0;
      YK_HIP(hipMalloc(&g->tile[e], need));
      g->tile_cap[e] = need;
    }
    if ((rc = ykgpu_render_async(c, &sub[e], g->tile[e], nullptr))) return rc;
  }
  // 2. each tile into rows e, e + k, e + 2k, ... of the caller's image (ordered after its render
  //    on the entry's stream)
  for (uint32_t e = 0; e < k; ++e) {
    if (!rows[e]) continue;
    ykgpu_context* c = g->ctx[e];
    YK_HIP(hipSetDevice(c->device));
    YK_HIP(hipMemcpy2DAsync(rgb_host + e * row_bytes, row_bytes * k, g->tile[e], row_bytes, row_bytes, rows[e],
                            hipMemcpyDeviceToHost, c->stream));
  }
  yk_render_stats tot{};
  for (uint32_t e = 0; e < k; ++e) {
    g->st[e] = yk_render_stats{};
    if (!rows[e]) continue;
    ykgpu_context* c = g->ctx[e];
    YK_HIP(hipSetDevice(c->device));
    YK_HIP(hipStreamSynchronize(c->stream));
    if ((rc = finish_stats(c))) return rc;
    g->st[e] = c->stats;
    const yk_render_stats& s = c->stats;
    tot.samples += s.samples;
    tot.segments += s.segments;
    tot.sphere_tests += s.sphere_tests;
    tot.sqrt_calls += s.sqrt_calls;
    tot.mt_fallbacks += s.mt_fallbacks;
    tot.node_visits += s.node_visits;
    tot.linear_scans += s.linear_scans;
    tot.newton_calls += s.newton_calls;
    tot.newton_iters += s.newton_iters;
    for (int q = 0; q < 8; ++q) tot.work[q] += s.work[q];
    tot.launches += s.launches;
    tot.grid_blocks = std::max(tot.grid_blocks, s.grid_blocks);
    tot.kernel_ms = std::max(tot.kernel_ms, s.kernel_ms);
    tot.render_busy_ms = std::max(tot.render_busy_ms, s.render_busy_ms);
    tot.warmup_ms = std::max(tot.warmup_ms, s.warmup_ms);
    tot.resolve_ms = std::max(tot.resolve_ms, s.resolve_ms);
    tot.seed_key = s.seed_key;
    tot.device_bytes += s.device_bytes + g->tile_cap[e];
    tot.call_bytes += s.call_bytes + rows[e] * row_bytes;
    tot.sclk_mhz = std::max(tot.sclk_mhz, s.sclk_mhz);
    // (ABI 11) the largest launch of any entry, and every entry's memory-pressure shrinks
    tot.launch_spp = std::max(tot.launch_spp, s.launch_spp);
    tot.mem_shrinks += s.mem_shrinks;
  }
  tot.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  g->total = tot;
  return YK_OK;
}

int ykgpu_group_get_stats(ykgpu_group* g, int index, yk_render_stats* out) {
  if (!g || !out) return fail(YK_ERR_INVALID, "null argument");
  if (index == -1) {
    *out = g->total;
    return YK_OK;
  }
  if (index < 0 || (size_t)index >= g->ctx.size()) return fail(YK_ERR_INVALID, "entry index out of range");
  *out = g->st[index];
  return YK_OK;
}

int ykgpu_render_devices(const int* devices, uint32_t n_devices, const yk_sphere* spheres, uint32_t count,
                         const yk_camera* camera, const yk_render_params* p, uint8_t* rgb_host) {
  ykgpu_group* g = nullptr;
  int rc = ykgpu_group_create(devices, n_devices, &g);
  if (!rc) rc = ykgpu_group_set_scene(g, spheres, count, camera);
  if (!rc) rc = ykgpu_group_render(g, p, rgb_host);
  if (g) {
    const std::string msg = g_last_error;
    ykgpu_group_destroy(g);
    g_last_error = msg;
  }
  return rc;
}

}  // extern "C"
#endif  // YK_SPLIT != 2
