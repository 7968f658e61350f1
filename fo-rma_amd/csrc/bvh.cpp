// Host BVH build: binned SAH (12 bins on the centroid extent of the longest axis),
// leaves of at most kBvhLeafMax primitives, emitted depth-first with escape links.
#include "bvh.h"

#include <math.h>

#include <algorithm>

namespace fr {
namespace {

struct Box3 {
  float lo[3] = {INFINITY, INFINITY, INFINITY};
  float hi[3] = {-INFINITY, -INFINITY, -INFINITY};
  void grow(const float p[3]) {
    for (int k = 0; k < 3; ++k) {
      lo[k] = std::min(lo[k], p[k]);
      hi[k] = std::max(hi[k], p[k]);
    }
  }
  void grow(const Box3& b) {
    grow(b.lo);
    grow(b.hi);
  }
  bool empty() const { return !(lo[0] <= hi[0]); }
  double area() const {
    if (empty()) return 0.0;
    const double dx = hi[0] - lo[0], dy = hi[1] - lo[1], dz = hi[2] - lo[2];
    return 2.0 * (dx * dy + dy * dz + dz * dx);
  }
};

// World bounds of one primitive; false for primitives that never hit (stubs) or
// carry non-finite geometry (those stay out of the tree and can never be the winner
// of the list loop either: their tests compare NaN).
bool prim_bounds(const fr_prim& p, Box3& b) {
  const float* g = p.g;
  switch (p.kind) {
    case FR_SPHERE: {
      const float r = fabsf(g[3]);
      const float lo[3] = {g[0] - r, g[1] - r, g[2] - r}, hi[3] = {g[0] + r, g[1] + r, g[2] + r};
      b.grow(lo);
      b.grow(hi);
      break;
    }
    case FR_AABB:
      b.grow(g);
      b.grow(g + 3);
      break;
    case FR_OBB: {
      // centre +- sum_j |axis_j| * half_j per world axis
      for (int k = 0; k < 3; ++k) {
        const float e = fabsf(g[3 + k]) * g[12] + fabsf(g[6 + k]) * g[13] + fabsf(g[9 + k]) * g[14];
        b.lo[k] = g[k] - e;
        b.hi[k] = g[k] + e;
      }
      break;
    }
    case FR_TRIANGLE:
      b.grow(g);
      b.grow(g + 3);
      b.grow(g + 6);
      break;
    default:
      return false;
  }
  for (int k = 0; k < 3; ++k)
    if (!std::isfinite(b.lo[k]) || !std::isfinite(b.hi[k])) return false;
  return true;
}

struct Item {
  Box3 box;
  float c[3];  // centroid
  uint32_t index;
};

struct Builder {
  std::vector<Item>& items;
  std::vector<BvhNode>& nodes;
  float pad;

  uint32_t order_base = 0;  // leaf indices are absolute positions in the shared order array

  // Emits the subtree over items[begin, end) at nodes.size(); returns its node index.
  uint32_t build(uint32_t begin, uint32_t end) {
    const uint32_t at = static_cast<uint32_t>(nodes.size());
    nodes.push_back(BvhNode{});
    Box3 box, cbox;
    for (uint32_t i = begin; i < end; ++i) {
      box.grow(items[i].box);
      cbox.grow(items[i].c);
    }
    for (int k = 0; k < 3; ++k) {  // conservative padding
      nodes[at].lo[k] = box.lo[k] - pad;
      nodes[at].hi[k] = box.hi[k] + pad;
    }
    const uint32_t n = end - begin;
    uint32_t mid = begin;
    if (n > kBvhLeafMax) mid = split(begin, end, box, cbox);
    if (mid == begin || mid == end) {  // leaf
      if (n > kBvhLeafMax) {           // no useful split (coincident centroids): halve by index
        mid = begin + n / 2;
      } else {
        nodes[at].leaf = (n << 24) | (order_base + begin);
        nodes[at].escape = static_cast<uint32_t>(nodes.size());
        return at;
      }
    }
    build(begin, mid);
    build(mid, end);
    nodes[at].leaf = 0;
    nodes[at].escape = static_cast<uint32_t>(nodes.size());
    return at;
  }

  // Binned SAH split; returns the partition point, or begin if a leaf is cheaper.
  uint32_t split(uint32_t begin, uint32_t end, const Box3& box, const Box3& cbox) {
    int axis = 0;
    float ext = -1.0f;
    for (int k = 0; k < 3; ++k)
      if (cbox.hi[k] - cbox.lo[k] > ext) {
        ext = cbox.hi[k] - cbox.lo[k];
        axis = k;
      }
    if (!(ext > 0.0f)) return begin;
    constexpr int B = 12;
    Box3 bb[B];
    uint32_t bc[B] = {};
    const float lo = cbox.lo[axis], scale = B / ext;
    auto bin_of = [&](const Item& it) {
      int b = static_cast<int>((it.c[axis] - lo) * scale);
      return b < 0 ? 0 : (b >= B ? B - 1 : b);
    };
    for (uint32_t i = begin; i < end; ++i) {
      const int b = bin_of(items[i]);
      bb[b].grow(items[i].box);
      ++bc[b];
    }
    double left_area[B], best = INFINITY;
    uint32_t left_count[B];
    Box3 acc;
    uint32_t cnt = 0;
    for (int b = 0; b < B; ++b) {
      acc.grow(bb[b]);
      cnt += bc[b];
      left_area[b] = acc.area();
      left_count[b] = cnt;
    }
    Box3 racc;
    uint32_t rcnt = 0;
    int best_b = -1;
    for (int b = B - 1; b > 0; --b) {
      racc.grow(bb[b]);
      rcnt += bc[b];
      const double cost = left_area[b - 1] * left_count[b - 1] + racc.area() * rcnt;
      if (left_count[b - 1] && rcnt && cost < best) {
        best = cost;
        best_b = b;
      }
    }
    const uint32_t n = end - begin;
    if (best_b < 0) return begin;
    // leaf cost n * area against 1 traversal + the split's cost
    if (n <= kBvhLeafMax && best >= box.area() * n) return begin;
    auto it = std::partition(items.begin() + begin, items.begin() + end,
                             [&](const Item& x) { return bin_of(x) < best_b; });
    return static_cast<uint32_t>(it - items.begin());
  }
};

float scene_abs_max(const std::vector<fr_prim>& prims) {
  float m = 0.0f;
  for (const fr_prim& p : prims) {
    Box3 b;
    if (!prim_bounds(p, b)) continue;
    for (int k = 0; k < 3; ++k) m = std::max(m, std::max(fabsf(b.lo[k]), fabsf(b.hi[k])));
  }
  return m;
}

bool build_range(const std::vector<fr_prim>& prims, uint32_t begin, uint32_t end, float pad,
                 std::vector<BvhNode>& nodes, std::vector<uint32_t>& order) {
  std::vector<Item> items;
  items.reserve(end - begin);
  for (uint32_t i = begin; i < end; ++i) {
    Item it;
    if (!prim_bounds(prims[i], it.box)) continue;
    for (int k = 0; k < 3; ++k) it.c[k] = 0.5f * (it.box.lo[k] + it.box.hi[k]);
    it.index = i;
    items.push_back(it);
  }
  if (items.empty()) return false;
  // Leaf indices must fit the node's 24-bit field.
  if (order.size() + items.size() >= (1u << 24)) return false;
  Builder b{items, nodes, pad};
  b.order_base = static_cast<uint32_t>(order.size());
  b.build(0, static_cast<uint32_t>(items.size()));
  for (const Item& it : items) order.push_back(it.index);
  return true;
}

}  // namespace

bool build_bvh(const std::vector<fr_prim>& prims, uint32_t begin, uint32_t end, std::vector<BvhNode>& nodes,
               std::vector<uint32_t>& order) {
  // The cull must never reject a primitive whose own test accepts a hit: pad every box
  // by a margin far above the f32 error of a root or a slab distance at scene scale.
  const float pad = 1e-4f * scene_abs_max(prims) + 1e-4f;
  return build_range(prims, begin, end, pad, nodes, order);
}

bool build_segments(const std::vector<fr_prim>& prims, std::vector<BvhSegment>& segs, std::vector<BvhNode>& nodes,
                    std::vector<uint32_t>& order, bool force) {
  segs.clear();
  nodes.clear();
  order.clear();
  const uint32_t n = static_cast<uint32_t>(prims.size());
  uint32_t planes = 0;
  for (const fr_prim& p : prims) planes += p.kind == FR_PLANE;
  float cost = 0.0f;
  for (const fr_prim& p : prims)
    cost += p.kind == FR_TRIANGLE ? 2.5f : p.kind == FR_OBB ? 2.0f : (p.kind == FR_STUB ? 0.0f : 1.0f);
  if (planes > kBvhMaxPlanes || n == 0) return false;
  if (!force && (n < kBvhMinPrims || cost < kBvhMinCost)) return false;
  const float pad = 1e-4f * scene_abs_max(prims) + 1e-4f;
  uint32_t i = 0;
  while (i < n) {
    if (prims[i].kind == FR_PLANE) {
      segs.push_back(BvhSegment{1u, 0u, 0u, i});
      ++i;
      continue;
    }
    uint32_t j = i;
    while (j < n && prims[j].kind != FR_PLANE) ++j;
    const uint32_t first = static_cast<uint32_t>(nodes.size());
    if (!build_range(prims, i, j, pad, nodes, order) && nodes.size() != first) return false;
    const uint32_t last = static_cast<uint32_t>(nodes.size());
    if (last > first) segs.push_back(BvhSegment{0u, first, last, 0u});
    i = j;
  }
  return true;
}

}  // namespace fr
