// Host BVH build: full-sweep SAH (every centroid position on all three axes) with
// leaves of at most kBvhLeafMax primitives, object-median splits where the depth cap
// (kBvhStack) would otherwise be at risk, nodes holding both children's boxes.
#include "bvh.h"

#include <math.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

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

// internal levels a balanced split of n items needs: ceil(log2(ceil(n / leaf_max)))
uint32_t balanced_levels(uint32_t n, uint32_t leaf_max) {
  uint32_t leaves = (n + leaf_max - 1) / leaf_max, l = 0;
  while ((1u << l) < leaves) ++l;
  return l;
}

struct Builder {
  std::vector<Item>& items;
  std::vector<BvhNode>& nodes;
  float pad;
  uint32_t leaf_max;
  uint32_t slot_base;  // leaf slots are absolute positions in the shared order array

  Box3 bounds(uint32_t begin, uint32_t end, Box3* cbox) const {
    Box3 box;
    for (uint32_t i = begin; i < end; ++i) {
      box.grow(items[i].box);
      if (cbox) cbox->grow(items[i].c);
    }
    return box;
  }

  // Reference to the subtree over items[begin, end) at depth `depth`.
  uint32_t build(uint32_t begin, uint32_t end, uint32_t depth) {
    const uint32_t n = end - begin;
    // FR_BVH_CT = c (A/B): SAH termination with a node step costing c primitive tests: a node
    // of at most FR_BVH_LEAF_CAP (8) primitives becomes a leaf when testing them all costs no
    // more than the best split (c + the children's area-weighted counts); off: every node
    // of at most leaf_max primitives is a leaf and every larger one is split
    static const double ct = [] {
      const char* e = getenv("FR_BVH_CT");
      return e ? atof(e) : -1.0;
    }();
    static const uint32_t leaf_cap = [] {
      const char* e = getenv("FR_BVH_LEAF_CAP");
      const int v = e ? atoi(e) : 8;
      return static_cast<uint32_t>(v >= 1 && v <= static_cast<int>(kBvhLeafCountMax) ? v : 8);
    }();
    if (ct < 0.0 && n <= leaf_max) return bvh_leaf_ref(slot_base + begin, n);
    Box3 cbox;
    const Box3 box = bounds(begin, end, &cbox);
    if (ct >= 0.0 && n <= std::max(leaf_cap, leaf_max)) {
      if (n == 1) return bvh_leaf_ref(slot_base + begin, n);
      double best = INFINITY;
      for (int k = 0; k < 3; ++k) {
        if (!(cbox.hi[k] - cbox.lo[k] > 0.0f)) continue;
        double c = INFINITY;
        sweep_split(begin, end, k, &c);
        best = std::min(best, c);
      }
      const double a = box.area();
      if (!(a > 0.0) || a * n <= ct * a + best) return bvh_leaf_ref(slot_base + begin, n);
    }
    // SAH while the subtree can still be finished below the cap by balanced splits
    // (a median split at depth d with d + levels(n) = kBvhStack leaves the deepest
    // internal node at kBvhStack - 1)
    uint32_t mid = begin;
    if (depth + balanced_levels(n, leaf_max) < kBvhStack) mid = sah_split(begin, end, box, cbox);
    if (mid == begin || mid == end) mid = median_split(begin, end, cbox);
    const uint32_t at = static_cast<uint32_t>(nodes.size());
    nodes.push_back(BvhNode{});
    const Box3 l = bounds(begin, mid, nullptr), r = bounds(mid, end, nullptr);
    const uint32_t rl = build(begin, mid, depth + 1);
    const uint32_t rr = build(mid, end, depth + 1);
    BvhNode& nd = nodes[at];
    // conservative padding
    for (int k = 0; k < 3; ++k) {
      nd.a[k] = l.lo[k] - pad;
      nd.b[k] = l.hi[k] + pad;
    }
    nd.a[3] = r.lo[0] - pad;
    nd.b[3] = r.hi[0] + pad;
    nd.c[0] = r.lo[1] - pad;
    nd.c[1] = r.lo[2] - pad;
    nd.c[2] = r.hi[1] + pad;
    nd.c[3] = r.hi[2] + pad;
    nd.ref[0] = rl;
    nd.ref[1] = rr;
    return at;
  }

  // Object median on the longest centroid axis; halves by index when the centroids
  // coincide.
  uint32_t median_split(uint32_t begin, uint32_t end, const Box3& cbox) {
    int axis = 0;
    float ext = -1.0f;
    for (int k = 0; k < 3; ++k)
      if (cbox.hi[k] - cbox.lo[k] > ext) {
        ext = cbox.hi[k] - cbox.lo[k];
        axis = k;
      }
    const uint32_t mid = begin + (end - begin) / 2;
    if (ext > 0.0f)
      std::nth_element(items.begin() + begin, items.begin() + mid, items.begin() + end,
                       [&](const Item& x, const Item& y) { return x.c[axis] < y.c[axis]; });
    return mid;
  }

  // SAH split: on each axis the centroids sorted and the area x count cost evaluated at every
  // position; the cheapest of the three axes. C5 trace 45.6 ms, against 46.5 for the sweep on
  // the longest axis only (FR_BVH_AXES=1) and 51.3 for 12 bins on the longest axis (8 bins
  // 48.5, 16 bins 52.3: binned trees walked at very different speeds). FR_BVH_BINS=k (A/B):
  // k bins on the longest axis instead (0: object medians).
  uint32_t sah_split(uint32_t begin, uint32_t end, const Box3& box, const Box3& cbox) {
    (void)box;
    int axis = 0;
    float ext = -1.0f;
    for (int k = 0; k < 3; ++k)
      if (cbox.hi[k] - cbox.lo[k] > ext) {
        ext = cbox.hi[k] - cbox.lo[k];
        axis = k;
      }
    if (!(ext > 0.0f)) return begin;
    static const int B = [] {
      const char* e = getenv("FR_BVH_BINS");
      const int v = e ? atoi(e) : -1;
      return v >= 0 && v <= 64 ? v : -1;
    }();
    static const bool all_axes = [] {
      const char* e = getenv("FR_BVH_AXES");
      return !(e && atoi(e) == 1);
    }();
    if (B < 0) {
      if (!all_axes) return sweep_split(begin, end, axis, nullptr);
      double best = INFINITY;
      int best_axis = -1;
      for (int k = 0; k < 3; ++k) {
        if (!(cbox.hi[k] - cbox.lo[k] > 0.0f)) continue;
        double cost = INFINITY;
        sweep_split(begin, end, k, &cost);
        if (cost < best) {
          best = cost;
          best_axis = k;
        }
      }
      return best_axis < 0 ? begin : sweep_split(begin, end, best_axis, nullptr);
    }
    if (B < 2) return begin;
    return binned_split(begin, end, cbox, axis, ext, B);
  }

  // items[begin, end) sorted by centroid on `axis` (ties by list index: deterministic);
  // returns the least-cost partition point (begin if none), its cost in *cost_out if given
  uint32_t sweep_split(uint32_t begin, uint32_t end, int axis, double* cost_out) {
    std::sort(items.begin() + begin, items.begin() + end, [&](const Item& x, const Item& y) {
      return x.c[axis] < y.c[axis] || (x.c[axis] == y.c[axis] && x.index < y.index);
    });
    const uint32_t n = end - begin;
    std::vector<double> right(n + 1, 0.0);
    Box3 acc;
    for (uint32_t i = n; i > 0; --i) {
      acc.grow(items[begin + i - 1].box);
      right[i - 1] = acc.area();
    }
    Box3 lacc;
    double best = INFINITY;
    uint32_t best_i = 0;
    for (uint32_t i = 1; i < n; ++i) {
      lacc.grow(items[begin + i - 1].box);
      const double cost = lacc.area() * i + right[i] * (n - i);
      if (cost < best) {
        best = cost;
        best_i = i;
      }
    }
    if (cost_out) *cost_out = best;
    return best_i ? begin + best_i : begin;
  }

  uint32_t binned_split(uint32_t begin, uint32_t end, const Box3& cbox, int axis, float ext, int B) {
    Box3 bb[64];
    uint32_t bc[64] = {};
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
    double left_area[64], best = INFINITY;
    uint32_t left_count[64];
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
    if (best_b < 0) return begin;
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

// Builds the tree over the boundable primitives of prims[begin, end); `root` is its
// reference (kBvhEnd when none is boundable). False if it cannot be encoded.
bool build_range(const std::vector<fr_prim>& prims, uint32_t begin, uint32_t end, float pad,
                 std::vector<BvhNode>& nodes, std::vector<uint32_t>& order, uint32_t& root) {
  std::vector<Item> items;
  items.reserve(end - begin);
  for (uint32_t i = begin; i < end; ++i) {
    Item it;
    if (!prim_bounds(prims[i], it.box)) continue;
    for (int k = 0; k < 3; ++k) it.c[k] = 0.5f * (it.box.lo[k] + it.box.hi[k]);
    it.index = i;
    items.push_back(it);
  }
  root = kBvhEnd;
  if (items.empty()) return true;
  const uint32_t n = static_cast<uint32_t>(items.size());
  // leaves of kBvhLeafMax, larger only when the balanced depth would not fit the stack
  // Leaves of 2 for lists with boxes, triangles or oriented boxes (their tests cost more
  // than a node step: scene_04 43.0 -> 38.4 ms, scene_05, _02, _06 1-2 % faster), 4 for
  // sphere-only lists (C5: 62.5 ms at 4, 63.0 at 2, 67.8 at 1).
  bool spheres_only = true;
  for (uint32_t i = begin; i < end; ++i) spheres_only = spheres_only && prims[i].kind == FR_SPHERE;
  uint32_t leaf_max = spheres_only ? kBvhLeafMax : kBvhLeafMax / 2u;
  if (const char* e = getenv("FR_BVH_LEAF"))  // A/B: primitives per leaf (1..16)
    if (atoi(e) >= 1 && atoi(e) <= static_cast<int>(kBvhLeafCountMax)) leaf_max = static_cast<uint32_t>(atoi(e));
  while (balanced_levels(n, leaf_max) >= kBvhStack && leaf_max < kBvhLeafCountMax) leaf_max *= 2;
  if (balanced_levels(n, leaf_max) >= kBvhStack) return false;
  if (order.size() + n + kBvhLeafCountMax >= (1u << kBvhSlotBits)) return false;
  if (nodes.size() + n >= kBvhLeaf) return false;
  Builder b{items, nodes, pad, leaf_max, static_cast<uint32_t>(order.size())};
  root = b.build(0, n, 0);
  for (const Item& it : items) order.push_back(it.index);
  return true;
}

uint32_t depth_of(const std::vector<BvhNode>& nodes, uint32_t ref, uint32_t depth) {
  if (ref >= kBvhLeaf) return 0;
  const BvhNode& nd = nodes[ref];
  return std::max({depth, depth_of(nodes, nd.ref[0], depth + 1), depth_of(nodes, nd.ref[1], depth + 1)});
}

}  // namespace

bool build_segments(const std::vector<fr_prim>& prims, std::vector<BvhSegment>& segs, std::vector<BvhNode>& nodes,
                    std::vector<uint32_t>& order, bool force, float* extent) {
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
  // The cull must never reject a primitive whose own test accepts a hit: pad every box
  // by a margin far above the f32 error of a root or a slab distance at scene scale.
  const float ext = scene_abs_max(prims);
  if (extent) *extent = ext;
  const float pad = 1e-4f * ext + 1e-4f;
  uint32_t i = 0;
  while (i < n) {
    if (prims[i].kind == FR_PLANE) {
      segs.push_back(BvhSegment{1u, kBvhEnd, 0u, i});
      ++i;
      continue;
    }
    uint32_t j = i;
    while (j < n && prims[j].kind != FR_PLANE) ++j;
    uint32_t root = kBvhEnd;
    if (!build_range(prims, i, j, pad, nodes, order, root)) return false;
    if (root != kBvhEnd) segs.push_back(BvhSegment{0u, root, 0u, 0u});
    i = j;
  }
  return true;
}

uint32_t bvh_max_depth(const std::vector<BvhSegment>& segs, const std::vector<BvhNode>& nodes) {
  uint32_t d = 0;
  for (const BvhSegment& s : segs)
    if (!s.plane) d = std::max(d, depth_of(nodes, s.root, 0));
  return d;
}

}  // namespace fr
