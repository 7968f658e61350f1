// Bounding volume hierarchy over a scene's primitives.
//
// A binary BVH whose nodes carry both children's boxes ("child boxes in the parent"):
// one 64-B fetch gives a lane two independent box tests; it steps into the nearer child
// it enters and keeps the other on a short per-lane stack in LDS. Leaves are referenced
// inline by the parent (first leaf slot, count) and their primitives' records are
// stored in leaf order, so a leaf costs no index hop. Used only as a conservative cull
// in front of the primitives' own tests; the closest-hit result is the same as the
// list-order loop (tracer.rs:195-200) because every primitive's candidate t does not
// depend on t_max and exact ties are broken by list index (render.hip, the BVH hit
// loop), whatever order the leaves are visited in.
#ifndef FR_BVH_H
#define FR_BVH_H

#include <stdint.h>

#if !defined(__HIPCC_RTC__)  // the constants below are also read by the run-time kernel build
#include <vector>

#include "../../include/forma_rt.h"
#else
#include "forma_rt.h"
#endif

namespace fr {

// Child reference: an internal node index (< kBvhLeaf), a leaf
// kBvhLeaf | (count - 1) << kBvhSlotBits | first slot, or kBvhEnd.
constexpr uint32_t kBvhLeaf = 0x80000000u;
constexpr uint32_t kBvhEnd = 0xFFFFFFFFu;
constexpr uint32_t kBvhSlotBits = 27;      // leaf slots < 2^27
constexpr uint32_t kBvhLeafCountMax = 16;  // count field: 4 bits
constexpr uint32_t bvh_leaf_ref(uint32_t first, uint32_t count) {
  return kBvhLeaf | ((count - 1u) << kBvhSlotBits) | first;
}

struct BvhNode {
  float a[4];       // left lo x y z, right lo x
  float b[4];       // left hi x y z, right hi x
  float c[4];       // right lo y z, right hi y z
  uint32_t ref[2];  // left, right child
  uint32_t pad[2];
};
static_assert(sizeof(BvhNode) == 64, "BvhNode is four float4");

constexpr uint32_t kBvhLeafMax = 4;    // primitives per leaf of sphere-only lists (2 for others; more only for huge scenes)
// The in-order loop (wave-uniform, scalar loads) beats the per-lane walk only for small
// lists: weight box / sphere 1, oriented box 2, triangle 2.5. Measured at 1080p
// (tools/bvh_threshold.sh): 43 mixed prims (scene_01) 38 ms in order vs 55 BVH; 50
// spheres 6.4 vs 5.1; 50 oriented boxes 17.9 vs 9.4; 74 (scene_05) 32.6 vs 27.1.
constexpr uint32_t kBvhMinPrims = 48;  // smaller scenes keep the in-order loop
constexpr float kBvhMinCost = 48.0f;
// Traversal stack entries per lane (LDS). The builder keeps every internal node at
// depth < kBvhStack (median splits where SAH would go deeper), and a lane holds at most
// one entry per internal node on its current path.
constexpr uint32_t kBvhStack = 16;

// The closest-hit list cut at its planes: runs of consecutive non-plane primitives (one
// BVH each) and single planes, in list order. A plane hit ignores t_max and may leave
// a stale record (plane.rs:24-44), so planes are tested one by one where they stand.
struct BvhSegment {
  uint32_t plane;  // 1: a plane, prims index `prim`; 0: a run
  uint32_t root;   // run: root reference (kBvhEnd: nothing boundable)
  uint32_t pad;
  uint32_t prim;
};
static_assert(sizeof(BvhSegment) == 16, "BvhSegment is one uint4");

constexpr uint32_t kBvhMaxPlanes = 32;  // more planes: the in-order loop

#if !defined(__HIPCC_RTC__)
// Segments, nodes and the leaf-order primitive list (`order[slot]` = list index) for a
// scene; false if the scene is too small, has too many planes or is too large for the
// reference encoding. `force` drops the size and cost thresholds (A/B runs).
// `extent` (if given) receives the largest |coordinate| of any primitive's bounds: the
// boxes are padded by 1e-4 * (extent + 1).
bool build_segments(const std::vector<fr_prim>& prims, std::vector<BvhSegment>& segs, std::vector<BvhNode>& nodes,
                    std::vector<uint32_t>& order, bool force = false, float* extent = nullptr);
#endif

// Ray origins the node cull is conservative for: |o| <= kBvhOriginReach * (extent + 1)
// (the kernel's fused node slabs add |o| 2^-24 to a slab distance; the padding allows
// 2^24 * 1e-4 = 1677 times that). A camera farther out renders with the in-order loop.
constexpr float kBvhOriginReach = 100.0f;
// The node cull's reciprocal direction is clamped to [-kBvhInvClamp, kBvhInvClamp]: a
// zero direction component (inv = +-inf) would make fma(lo, inv, -o inv) NaN. A clamped
// slab is still conservative: a hit inside a box padded by >= 1e-4 keeps that axis's
// slab >= 1e-4 * 2^100 ~ 1e26 wide, and |o| 2^100 stays finite.
constexpr float kBvhInvClamp = 0x1p100f;

#if !defined(__HIPCC_RTC__)
// Largest internal-node depth of the trees (root = 0): below kBvhStack by construction.
uint32_t bvh_max_depth(const std::vector<BvhSegment>& segs, const std::vector<BvhNode>& nodes);
#endif

}  // namespace fr

#endif
