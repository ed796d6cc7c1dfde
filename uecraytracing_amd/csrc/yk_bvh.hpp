// yk_bvh.hpp — bounding volume hierarchy over the world's spheres (host build, device layout).
//
// The BVH only CULLS: it never decides a hit.  The closest-hit rule of the reference
// (hittable_list.hpp:32-58: minimum root, exact ties to the later tuple index) is applied to
// the surviving candidates with the reference's exact arithmetic, so the result is identical to
// the ordered linear scan whatever the tree looks like.  Culling is conservative:
//   * boxes are the spheres' bounds grown by kDelta and rounded outward to float;
//   * kDelta >= 2^-21 * origin_bound, so a ray origin rounded to float moves by less than the
//     growth, and every root the exact test can return lies inside the grown box;
//   * slab distances computed in float are compared with a 2^-20 relative slack.
// Rays whose origin lies beyond origin_bound use the exact linear scan instead.
#pragma once

#include <cstdint>
#include <vector>

namespace ykbvh {

// Binary node, both children's boxes stored in the parent: 64 bytes, 4 x 16-B loads.
// child >= 0: inner node index; child < 0: leaf, ~child = first << 4 | count (count 1..15).
struct alignas(16) Node {
  float lo_x[2], lo_y[2], lo_z[2];
  float hi_x[2], hi_y[2], hi_z[2];
  int32_t child[2];
  int32_t pad[2];
};
static_assert(sizeof(Node) == 64, "Node layout");

// 4-wide device node (160 bytes), built by wide_nodes() by collapsing the binary tree: each slot
// whose child is an inner node is replaced by that node's two children, the largest surface
// area first, until the node has 4 slots or only leaves.  Per axis, the 4 slots' planes as
// [lo x4][hi x4][lo x4]: a ray with 1/d >= 0 reads (near x4, far x4) at bytes (0, 16) of the
// axis, a ray with 1/d < 0 at (16, 32) — one 16-byte read per plane set returns the planes
// already ordered, so the slab test needs no min/max (rounding is monotonic, so the selection
// equals min/max of the two products).  child >= 0 is
// the BYTE OFFSET of an inner WideNode, < 0 a leaf code; an unused slot has an empty box
// (lo = +3e38, hi = -3e38: near > far for any ray) and the empty leaf code ~0 (no spheres).
// The culling per slot is the binary node's (same planes, same rounding): DESIGN.md §4 holds.
struct alignas(16) WideNode {
  float x[12], y[12], z[12];
  int32_t child[4];
};
static_assert(sizeof(WideNode) == 160, "WideNode layout");
constexpr int32_t kEmptyLeaf = ~0;  // leaf code with no spheres

// render<float>'s sphere test (sphere.hpp:25-48 evaluated in float) near tangency: a root it
// accepts puts the exact point o + r d within 2^-8.9 (|o - c| + |radius|) of the float sphere,
// hence within 2^-8.9 (r |d| + 2 |radius|).  FP32 trees grow each sphere's box
// by 2 kF32Cone |radius| on top of delta, and the FP32 kernel widens every ray into a cone of
// slope kF32Cone |d|: 1.87x the bound.
constexpr float kF32Cone = 0x1p-8f * (1.0f + 0x1p-10f);
// A sphere that every hit distance stays within kF32BigReach radii of (kF32BigReach |radius| >=
// sqrt(3) origin_bound + |c| + |radius|) needs far less: the bound's quadratic form,
// 72.7 u (t^2 |d|^2 / R + 2 t |d| + 2 R) with u = 2^-24, stays below
// kF32Cone t |d| + kF32BigGrow |radius| there (3.5x margin on 72.7 u).  The RTIOW ground sphere
// (r = 1000) then grows by 0.03 instead of 7.8.
constexpr double kF32BigGrow = 0x1p-15;
constexpr double kF32BigReach = 192.0;

struct Built {
  std::vector<Node> nodes;      // nodes[0] is the root when root >= 0
  std::vector<uint32_t> order;  // leaf slots → original sphere index (tuple order)
  int32_t root = 0;             // root code (a leaf code when the scene has one leaf)
  uint32_t depth = 0;           // longest root-to-leaf path (inner nodes)
  double origin_bound = 0;      // |o|_inf above which a ray uses the exact linear scan
  float delta = 0;              // box growth
};

struct Options {
  uint32_t max_leaf = 2;  // spheres per leaf (<= 15); callers pick per kernel
  int bins = 16;          // SAH bins per split
  bool all_axes = false;  // SAH over all three axes (false: the longest centroid axis only)
  double radius_grow = 0; // extra box growth per unit |radius| (FP32 trees: 2 kF32Cone)
  bool f32_big = false;   // FP32 trees: kF32BigGrow for spheres within kF32BigReach radii
};

// centers: 3 doubles per sphere; radii may be negative (hollow shells: |r| is used).
Built build(const double* centers, const double* radii, uint32_t n, double camera_extent,
            const Options& opt = Options());
// 4-wide nodes (DFS order, root first), the root code in that encoding, and the wide depth
// (inner nodes on the longest root-to-leaf path).
std::vector<WideNode> wide_nodes(const Built& b, int32_t* root_code, uint32_t* wide_depth);
constexpr uint32_t kMaxDepth = 32;  // traversal stack capacity (device, LDS)

}  // namespace ykbvh
