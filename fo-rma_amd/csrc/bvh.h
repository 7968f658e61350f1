// Bounding volume hierarchy over a scene's primitives.
//
// A threaded ("stackless") binary BVH in depth-first order: an internal node's first
// child is the next node, and every node carries an escape index, the node after its
// subtree. A lane walks it with one index: on a box miss or after a leaf it jumps to
// `escape`, otherwise it steps to the next node. No stack, so no LDS or registers per
// level. Used only as a conservative cull in front of the primitives' own tests; the
// closest-hit result is the same as the list-order loop (tracer.rs:195-200) because
// every primitive's candidate t does not depend on t_max and exact ties are broken by
// list index (render.hip, the BVH hit loop).
#ifndef FR_BVH_H
#define FR_BVH_H

#include <stdint.h>

#include <vector>

#include "../../include/forma_rt.h"

namespace fr {

struct BvhNode {
  float lo[3];
  uint32_t escape;  // next node when this box is missed or this leaf is done
  float hi[3];
  uint32_t leaf;    // 0: internal (first child = this + 1); else (count << 24) | first
};
static_assert(sizeof(BvhNode) == 32, "BvhNode is two float4");

constexpr uint32_t kBvhLeafMax = 4;      // primitives per leaf
constexpr uint32_t kBvhMinPrims = 64;    // smaller scenes keep the in-order loop
// The in-order loop (wave-uniform, scalar loads) beats a divergent per-lane walk until
// a segment's tests cost enough: weight box / sphere 1, oriented box 2, triangle 2.5
// (measured: 217 boxes 93 ms in order vs 124 ms BVH; 156 triangles 49 ms vs 19 ms).
constexpr float kBvhMinCost = 300.0f;

// Builds the BVH over prims[begin, end) (stubs are left out: they never hit), appending
// its nodes to `nodes` and its leaf primitive indices (global) to `order`; escape and
// leaf indices are absolute. Returns false (appending nothing) if no primitive of the
// range can be bounded.
bool build_bvh(const std::vector<fr_prim>& prims, uint32_t begin, uint32_t end, std::vector<BvhNode>& nodes,
               std::vector<uint32_t>& order);

// The closest-hit list cut at its planes: runs of consecutive non-plane primitives (one
// BVH each) and single planes, in list order. A plane hit ignores t_max and may leave
// a stale record (plane.rs:24-44), so planes are tested one by one where they stand.
struct BvhSegment {
  uint32_t plane;       // 1: a plane, prims index `prim`; 0: a run with nodes [first, end)
  uint32_t first, end;  // node range of the run's tree (end == first: nothing boundable)
  uint32_t prim;
};
static_assert(sizeof(BvhSegment) == 16, "BvhSegment is one uint4");

constexpr uint32_t kBvhMaxPlanes = 32;  // more planes: the in-order loop

// Segments and trees for a scene; false if the scene is too small or has too many planes
// (`force` drops the size and cost thresholds, for A/B runs).
bool build_segments(const std::vector<fr_prim>& prims, std::vector<BvhSegment>& segs, std::vector<BvhNode>& nodes,
                    std::vector<uint32_t>& order, bool force = false);

}  // namespace fr

#endif
