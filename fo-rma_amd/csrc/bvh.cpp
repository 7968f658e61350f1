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
        nodes[at].leaf = (n << 24) | begin;
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

}  // namespace

bool build_bvh(const std::vector<fr_prim>& prims, std::vector<BvhNode>& nodes, std::vector<uint32_t>& order) {
  nodes.clear();
  order.clear();
  std::vector<Item> items;
  items.reserve(prims.size());
  float scene_abs = 0.0f;
  for (uint32_t i = 0; i < prims.size(); ++i) {
    Item it;
    if (!prim_bounds(prims[i], it.box)) continue;
    for (int k = 0; k < 3; ++k) {
      it.c[k] = 0.5f * (it.box.lo[k] + it.box.hi[k]);
      scene_abs = std::max(scene_abs, std::max(fabsf(it.box.lo[k]), fabsf(it.box.hi[k])));
    }
    it.index = i;
    items.push_back(it);
  }
  if (items.empty()) return false;
  // The cull must never reject a primitive whose own test accepts a hit: pad every box
  // by a margin far above the f32 error of a root or a slab distance at scene scale.
  Builder b{items, nodes, 1e-4f * scene_abs + 1e-4f};
  b.build(0, static_cast<uint32_t>(items.size()));
  order.resize(items.size());
  for (size_t i = 0; i < items.size(); ++i) order[i] = items[i].index;
  return true;
}

}  // namespace fr
