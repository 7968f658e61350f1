// Host BVH build: full-sweep SAH (every centroid position on all three axes) with
// leaves of at most kBvhLeafMax primitives, object-median splits where the depth cap
// (kBvhStack) would otherwise be at risk, nodes holding both children's boxes. O(n log n):
// the three axis orders are sorted once and kept sorted per node by stable partitions.
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

// The builder keeps, per axis, the items' ids sorted by (centroid on that axis, list index)
// within every open node's range. A node's three SAH sweeps then read their orders without
// sorting, and a split stable-partitions the other two axes' ids by side, so each level costs
// O(n) (the round-5 builder sorted every node's items four times: 1.06 s for 150k spheres,
// 39.5 ms for C5; this one builds the same trees, checked by digest in
// tests/test_host_sanitizers.py). A leaf's slots list its items in the order of the axis
// its parent split on (list order for a root leaf).
struct Builder {
  const std::vector<Item>& items;  // by item id
  std::vector<BvhNode>& nodes;
  std::vector<uint32_t>& slots;    // item id per leaf slot, relative to slot 0 of this tree
  float pad;
  uint32_t leaf_max;
  uint32_t leaf_cap = kBvhLeafCountMax;  // SAH-terminated leaves: at most this many items
  double sah_ct = 0.0;                   // node step cost in leaf tests (0: leaves of leaf_max)
  uint32_t slot_base;  // leaf slots are absolute positions in the shared order array
  std::vector<uint32_t> idx[3];
  std::vector<uint8_t> on_left;  // by item id, scratch of one split
  std::vector<uint32_t> tmp;
  std::vector<double> right;

  Builder(const std::vector<Item>& it, std::vector<BvhNode>& nd, std::vector<uint32_t>& sl, float p, uint32_t lm,
          uint32_t base)
      : items(it), nodes(nd), slots(sl), pad(p), leaf_max(lm), slot_base(base) {
    const uint32_t n = static_cast<uint32_t>(items.size());
    for (int k = 0; k < 3; ++k) {
      idx[k].resize(n);
      for (uint32_t i = 0; i < n; ++i) idx[k][i] = i;
      std::sort(idx[k].begin(), idx[k].end(), [&](uint32_t x, uint32_t y) {
        return items[x].c[k] < items[y].c[k] || (items[x].c[k] == items[y].c[k] && items[x].index < items[y].index);
      });
    }
    on_left.assign(n, 0);
    tmp.resize(n);
    right.resize(n + 1);
    slots.assign(n, 0);
  }

  Box3 bounds(const uint32_t* ids, uint32_t n, Box3* cbox) const {
    Box3 box;
    for (uint32_t i = 0; i < n; ++i) {
      box.grow(items[ids[i]].box);
      if (cbox) cbox->grow(items[ids[i]].c);
    }
    return box;
  }

  // Reference to the subtree over range [begin, end) at depth `depth`; `pa` is the axis the
  // parent split on (-1 at the root: list order).
  uint32_t build(uint32_t begin, uint32_t end, uint32_t depth, int pa) {
    const uint32_t n = end - begin;
    if (n <= leaf_max) return leaf(begin, n, pa);
    Box3 cbox;
    const Box3 box = bounds(idx[0].data() + begin, n, &cbox);
    // SAH while the subtree can still be finished below the cap by balanced splits
    // (a median split at depth d with d + levels(n) = kBvhStack leaves the deepest
    // internal node at kBvhStack - 1)
    int axis = -1;
    uint32_t mid = begin;
    double split = INFINITY;  // the chosen split's sum of (side area x count)
    if (depth + balanced_levels(n, leaf_max) < kBvhStack) sah_split(begin, end, cbox, &axis, &mid, &split);
    // SAH termination (sah_ct > 0): a leaf of up to leaf_cap items where testing them all
    // costs no more than a node step (sah_ct leaf tests) plus the split's expected tests
    if (sah_ct > 0.0 && n <= leaf_cap && split < INFINITY && box.area() > 0.0 &&
        static_cast<double>(n) <= sah_ct + split / box.area())
      return leaf(begin, n, pa);
    if (mid == begin || mid == end) median_split(begin, end, cbox, &axis, &mid);
    // ids of the left side first on every axis, each side in its axis order
    for (uint32_t i = begin; i < end; ++i) on_left[idx[axis][i]] = i < mid;
    for (int k = 0; k < 3; ++k) {
      if (k == axis) continue;
      uint32_t l = begin, r = 0;
      for (uint32_t i = begin; i < end; ++i) {
        const uint32_t id = idx[k][i];
        if (on_left[id])
          idx[k][l++] = id;
        else
          tmp[r++] = id;
      }
      std::copy(tmp.begin(), tmp.begin() + r, idx[k].begin() + l);
    }
    const uint32_t at = static_cast<uint32_t>(nodes.size());
    nodes.push_back(BvhNode{});
    const Box3 l = bounds(idx[axis].data() + begin, mid - begin, nullptr);
    const Box3 r = bounds(idx[axis].data() + mid, end - mid, nullptr);
    const uint32_t rl = build(begin, mid, depth + 1, axis);
    const uint32_t rr = build(mid, end, depth + 1, axis);
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

  // a leaf over range [begin, begin + n): its slots in the parent's split-axis order
  uint32_t leaf(uint32_t begin, uint32_t n, int pa) {
    if (pa < 0) {  // a root leaf keeps list order (ids are list-ordered)
      for (uint32_t i = 0; i < n; ++i) slots[begin + i] = begin + i;
    } else {
      for (uint32_t i = 0; i < n; ++i) slots[begin + i] = idx[pa][begin + i];
    }
    return bvh_leaf_ref(slot_base + begin, n);
  }

  static int longest(const Box3& cbox, float* ext_out) {
    int axis = 0;
    float ext = -1.0f;
    for (int k = 0; k < 3; ++k)
      if (cbox.hi[k] - cbox.lo[k] > ext) {
        ext = cbox.hi[k] - cbox.lo[k];
        axis = k;
      }
    *ext_out = ext;
    return axis;
  }

  // Object median on the longest centroid axis (ties by list index); halves in list order
  // when the centroids coincide (every axis order is then list order).
  void median_split(uint32_t begin, uint32_t end, const Box3& cbox, int* axis, uint32_t* mid) {
    float ext;
    const int a = longest(cbox, &ext);
    *axis = ext > 0.0f ? a : 0;
    *mid = begin + (end - begin) / 2;
  }

  // SAH split: on each axis the cost (area x count per side) at every position of the
  // centroid order; the cheapest of the three axes (the first on ties), at its first
  // cheapest position. C5 trace 45.6 ms, against 46.5 for the sweep on the longest axis only
  // and 51.3 for 12 bins on the longest axis (8 bins 48.5, 16 bins 52.3: binned trees walked
  // at very different speeds; profiles/AB_LOG.md).
  void sah_split(uint32_t begin, uint32_t end, const Box3& cbox, int* axis, uint32_t* mid, double* cost_out) {
    float ext;
    (void)longest(cbox, &ext);
    if (!(ext > 0.0f)) return;
    double best = INFINITY;
    for (int k = 0; k < 3; ++k) {
      if (!(cbox.hi[k] - cbox.lo[k] > 0.0f)) continue;
      double cost = INFINITY;
      const uint32_t i = sweep(begin, end, k, &cost);
      if (cost < best && i) {
        best = cost;
        *axis = k;
        *mid = begin + i;
      }
    }
    *cost_out = best;
  }

  // the least-cost partition position of the range in axis k's order (0 if none)
  uint32_t sweep(uint32_t begin, uint32_t end, int k, double* cost_out) {
    const uint32_t n = end - begin;
    const uint32_t* ids = idx[k].data() + begin;
    Box3 acc;
    for (uint32_t i = n; i > 0; --i) {
      acc.grow(items[ids[i - 1]].box);
      right[i - 1] = acc.area();
    }
    Box3 lacc;
    double best = INFINITY;
    uint32_t best_i = 0;
    for (uint32_t i = 1; i < n; ++i) {
      lacc.grow(items[ids[i - 1]].box);
      const double cost = lacc.area() * i + right[i] * (n - i);
      if (cost < best) {
        best = cost;
        best_i = i;
      }
    }
    *cost_out = best;
    return best_i;
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
  std::vector<uint32_t> slots;
  Builder b(items, nodes, slots, pad, leaf_max, static_cast<uint32_t>(order.size()));
  if (const char* e = getenv("FR_BVH_SAH_CT")) b.sah_ct = atof(e);  // A/B
  if (const char* e = getenv("FR_BVH_LEAF_CAP"))
    if (atoi(e) >= 1 && atoi(e) <= static_cast<int>(kBvhLeafCountMax)) b.leaf_cap = static_cast<uint32_t>(atoi(e));
  root = b.build(0, n, 0, -1);
  for (uint32_t id : slots) order.push_back(items[id].index);
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
