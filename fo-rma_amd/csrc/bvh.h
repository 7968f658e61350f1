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

// Builds the BVH over prims (stubs are left out: they never hit). `order` receives the
// primitive indices in leaf order. Returns false (and leaves both empty) if no
// primitive can be bounded.
bool build_bvh(const std::vector<fr_prim>& prims, std::vector<BvhNode>& nodes, std::vector<uint32_t>& order);

}  // namespace fr

#endif
