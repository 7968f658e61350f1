// render.hip — the gfx950 path-tracing megakernel and its host driver.
//
// Replaces cpu_ray_tracer/tracer.rs:160-219 (save_image + recursive get_color)
// and the shapes/ hit/scatter code it calls. A persistent grid pulls work items
// (one pixel's 16-sample RNG block) from a global counter; every lane holds one path
// segment per loop iteration and a lane whose path ends starts its next sample at
// once (path regeneration), so lanes never wait for each other's pixels. Each
// sample's colour goes to a per-sample buffer that sum_kernel adds per pixel in
// sample order, exactly as `col = col + get_color(...)` does (tracer.rs:170-175).
// The attenuation product is unwound right-to-left from a per-lane LDS stack,
// reproducing the recursion's association a0*(a1*(...*terminal)) bit for bit.
//
// Closest hit: small scenes test primitive i on every lane at once (wave-uniform:
// the kind switch is a scalar branch, records arrive by scalar loads); large ones
// walk a BVH per lane (LDS stack), cut at the planes (bvh.h). Layout and rooflines:
// DESIGN.md §4-§5.
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <chrono>
#include <cmath>
#include <algorithm>
#include <string>
#include <thread>
#include <type_traits>

#include "bvh.h"
#include "internal.h"
#include "sum.h"
#include "trace_kernel.h"
#include "jit.h"
#include <atomic>

#define HIPCHK(call)                                                                      \
  do {                                                                                    \
    hipError_t e_ = (call);                                                               \
    if (e_ != hipSuccess)                                                                 \
      return fr::set_error(FR_EHIP, "%s failed: %s", #call, hipGetErrorString(e_));       \
  } while (0)

namespace fr {

// Sets a call's device and restores the caller's current device when the call returns,
// so an entry point never leaves torch (or any other caller) on another device.
struct DeviceGuard {
  int prev = -1;
  hipError_t err;
  explicit DeviceGuard(int d) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    err = hipSetDevice(d);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};
#define SET_DEVICE(d)               \
  fr::DeviceGuard dev_guard_((d));  \
  HIPCHK(dev_guard_.err)


// ABI layout, mirrored by ctypes (forma_rt.py) and the Rust binding
static_assert(sizeof(fr_prim) == 88, "fr_prim layout");
static_assert(sizeof(fr_camera) == 104, "fr_camera layout");
static_assert(sizeof(fr_params) == 40, "fr_params layout");
static_assert(sizeof(fr_stats) == 72, "fr_stats layout");

struct DeviceCopy {
  int device = -1;
  uint64_t version = 0;
  uint64_t uid = 0;  // process-unique per upload: names these exact records (fr_ctx's kernel cache)
  void* blob = nullptr;
  uint32_t n = 0;
  bool has_plane = false;
  uint32_t kinds = 0;  // bit k set if a primitive of kind k is present
  size_t off_mat = 0, off_cls = 0, off_att = 0;
  size_t off_rec = 0;
  size_t off_bvh = 0, off_bvh_order = 0, off_lrec = 0, off_segs = 0, off_runs = 0;
  uint32_t n_runs = 0;
  bool bvh_ok = false;  // segments and trees built (else the in-order loop only)
  float bvh_extent = 0; // largest |coordinate| of the primitives' bounds (bvh.h)
  uint32_t n_segs = 0;  // closest-hit segments: BVH runs and planes (bvh.h)
  // traversal-stack levels a lane can use: the trees' largest internal-node depth + 1 (a
  // lane at depth d holds at most d entries and writes the free one): the BVH launch's LDS
  uint32_t bvh_levels = kBvhStack;
  bool att_nonneg = true;  // every attenuation component finite and >= +0 (no -0)
  bool diffuse = true;     // no metal or dielectric scatter class (trace_kernel MAT = 1)
  // attenuation classes: the scene's distinct attenuations (bit patterns), when there are at
  // most kNibbleMaxPrims of them (else 0): BVH kernels with 8-B records store a path's
  // winners as classes (KScene::acls), and sum_nib_kernel reads this table instead of one
  // entry per primitive
  uint32_t n_aclass = 0;
  size_t off_acls = 0, off_acls_att = 0;
  std::vector<uint32_t> rec_words;  // the n 64-B records as uploaded (the scene-specialised build's constants)
};


static void fastdiv_magic(uint32_t d, uint32_t& m, uint32_t& shifts) {
  if (d < 1) d = 1;
  const uint32_t l = d == 1 ? 0u : 32u - static_cast<uint32_t>(__builtin_clz(d - 1));
  m = static_cast<uint32_t>(((static_cast<uint64_t>(1) << 32) * ((static_cast<uint64_t>(1) << l) - d)) / d + 1);
  shifts = (l < 1 ? l : 1u) | ((l > 0 ? l - 1 : 0u) << 1);
}


// Effective scatter class after each shape's fallback chain
// (sphere.rs:56-69: 0/1/2/3 else lambertian; plane.rs:48-59: 1 metal else lambertian).
static uint32_t scatter_class(const fr_prim& p) {
  if (p.kind == FR_STUB) return SC_NONE;
  if (p.kind == FR_PLANE) return p.material == FR_METAL ? SC_METAL : SC_LAMBERT;
  switch (p.material) {
    case FR_METAL: return SC_METAL;
    case FR_DIELECTRIC: return SC_DIELECTRIC;
    case FR_LIGHT: return SC_LIGHT;
    default: return SC_LAMBERT;
  }
}


// Sums the trace kernel's per-wave counters (KWork::wave_counters) into counters[0..2].
__global__ __launch_bounds__(256) void reduce_counters(const unsigned long long* __restrict__ wc, uint32_t waves,
                                                       unsigned long long* __restrict__ counters) {
  __shared__ unsigned long long part[3][256];
  unsigned long long v[3] = {0, 0, 0};
  for (uint32_t w = threadIdx.x; w < waves; w += 256)
    for (int k = 0; k < 3; ++k) v[k] += wc[3 * w + k];
  for (int k = 0; k < 3; ++k) part[k][threadIdx.x] = v[k];
  __syncthreads();
  for (uint32_t h = 128; h > 0; h >>= 1) {
    if (threadIdx.x < h)
      for (int k = 0; k < 3; ++k) part[k][threadIdx.x] += part[k][threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x < 3) atomicAdd(&counters[threadIdx.x], part[threadIdx.x][0]);  // passes on two streams
}

// ---- diagnostics kernels ---------------------------------------------------

__global__ void ops_kernel(int op, const float* a, const float* b, uint32_t n, float* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float x = a[i], y = b[i];
  float r;
  switch (op) {
    case 0: r = x + y; break;
    case 1: r = x - y; break;
    case 2: r = x * y; break;
    case 3: r = x / y; break;
    case 4: r = sqrtf(x); break;
    case 5: r = schlick(x, y); break;
    case 6: r = static_cast<float>(to_u8(x)); break;
    case 7: r = unit(V3{x, y, 1.0f}).x; break;
    case 8: r = 1.0f / x; break;
    case 9: r = div_rn(x, y, 1.0f / y); break;  // the kernel's jitter division
    case 10: r = recip_nr_ok(x) ? recip_nr(x) : 1.0f / x; break;
    case 11: r = fmax3_num(x, y, b[(i + 1) % n]); break;  // vs fmaxf(fmaxf(x, y), z)
    case 12: r = fmin3_num(x, y, b[(i + 1) % n]); break;  // vs fminf(fminf(x, y), z)
    case 17: r = fmin_num(fmin_num(x, y), b[(i + 1) % n]); break;  // chained v_min_f32
    case 13: r = fmax_num(fmax_num(x, y), b[(i + 1) % n]); break;  // chained v_max_f32
    case 14: {  // sky_t_fast against sky_t on the direction (x, y, z = b[i + 1]): 0 when equal bits
      const V3 dv{x, y, b[(i + 1) % n]};
      r = __uint_as_float(__float_as_uint(sky_t_fast(dv)) ^ __float_as_uint(sky_t(dv)));
      break;
    }
    case 15: r = sky_t_fast(V3{x, y, b[(i + 1) % n]}); break;
    case 16: {
      // sphere_root_fast against sphere_root: thread 16k reads a[16k..16k+10] = centre,
      // radius, origin, direction, t_max (t_min = 0.001). 0: same verdict and t bits;
      // 1: verdicts differ; 2: both hit with different t
      if (i % 16u != 0u || i + 16u > n) {
        r = 0.0f;
        break;
      }
      const float* q = a + i;
      const V3 c{q[0], q[1], q[2]}, o{q[4], q[5], q[6]}, dv{q[7], q[8], q[9]};
      const float aa = dot(dv, dv);
      float t0 = 0.0f, t1 = 0.0f;
      const bool h0 = sphere_root(c, q[3], o, dv, aa, 0.001f, q[10], t0);
      const bool h1 = sphere_root_fast(c, q[3], o, dv, aa, sphere_seg(aa), 0.001f, q[10], t1);
      r = h0 != h1 ? 1.0f : (h0 && __float_as_uint(t0) != __float_as_uint(t1)) ? 2.0f : 0.0f;
      break;
    }
    default: r = 0.0f;
  }
  out[i] = r;
}

// Exhaustive check of recip_nr (rcp + one FMA Newton step) against the correctly
// rounded 1.0f / x over x = [base, base + count): per exponent field (256 buckets) the
// number of results whose bits differ (NaN == NaN) and the first such input.
__global__ void recip_check_kernel(uint64_t base, uint64_t count, unsigned long long* bad, uint32_t* first) {
  const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
  for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < count; i += stride) {
    const uint32_t bits = static_cast<uint32_t>(base + i);
    const float x = __uint_as_float(bits);
    const float want = 1.0f / x, got = recip_nr(x);
    const bool same = __float_as_uint(want) == __float_as_uint(got) || (want != want && got != got);
    if (!same) {
      const uint32_t e = (bits >> 23) & 0xFFu;
      atomicAdd(&bad[e], 1ull);
      atomicMin(&first[e], bits);
    }
  }
}

// Exhaustive check of div_rn against the correctly rounded a / b over the mantissa
// space: the threads take every a = 1 + i 2^-23 (all 2^23 of [1, 2)), the loop every
// b = 1 + m 2^-23 with m in [b_base, b_base + b_count), y = RN(1 / b). Division by powers
// of two on either operand scales both results exactly while no intermediate leaves the
// normal range, so [1, 2) x [1, 2) covers every use (rt_core.h div_rn). bad[0] counts the
// pairs whose bits differ, first[0] holds the least (m << 23 | i) of them.
__global__ void div_check_kernel(uint32_t b_base, uint32_t b_count, unsigned long long* bad,
                                 unsigned long long* first) {
  // four a per thread (i + j 2^21), so that each y = 1.0f / b serves four pairs
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (1u << 21)) return;
  unsigned long long nbad = 0, fbad = ~0ull;
  for (uint32_t k = 0; k < b_count; ++k) {
    const uint32_t m = b_base + k;
    const float b = __uint_as_float(0x3F800000u | m);
    const float y = 1.0f / b;
#pragma unroll
    for (uint32_t j = 0; j < 4; ++j) {
      const uint32_t ia = i + (j << 21);
      const float a = __uint_as_float(0x3F800000u | ia);
      const float want = a / b, got = div_rn(a, b, y);
      if (__float_as_uint(want) != __float_as_uint(got)) {
        ++nbad;
        fbad = min(fbad, (static_cast<unsigned long long>(m) << 23) | ia);
      }
    }
  }
  if (nbad) {
    atomicAdd(bad, nbad);
    atomicMin(first, fbad);
  }
}

__global__ void rng_kernel(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, uint32_t* out) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  Rng r = rng_seed(seed, pixel, sample);
  for (uint32_t i = 0; i < n; ++i) out[i] = rng_next(r);
}

// ---- device scene copies ----------------------------------------------------

static size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

static int upload_scene(fr_scene* s, int device, DeviceCopy** out) {
  std::lock_guard<std::mutex> g(s->mu);
  for (DeviceCopy* c : s->copies)
    if (c->device == device) {
      if (c->version == s->version) {
        *out = c;
        return FR_OK;
      }
      HIPCHK(hipFree(c->blob));
      c->blob = nullptr;
    }
  DeviceCopy* c = nullptr;
  for (DeviceCopy* e : s->copies)
    if (e->device == device) c = e;
  if (!c) {
    c = new DeviceCopy();
    c->device = device;
    s->copies.push_back(c);
  }
  const uint32_t n = static_cast<uint32_t>(s->prims.size());
  const size_t m = n ? n : 1;  // never hand the kernel a null array
  // BVH runs between planes for scenes of kBvhMinPrims or more (bvh.h)
  std::vector<BvhSegment> bvh_segs;
  std::vector<BvhNode> bvh_nodes;
  std::vector<uint32_t> bvh_order;
  // FR_BVH=1 builds the BVH below the size/cost thresholds (A/B runs), FR_BVH=0 never uses it
  const char* bvh_env = getenv("FR_BVH");
  const bool force_bvh = bvh_env && strcmp(bvh_env, "1") == 0;
  float bvh_extent = 0.0f;
  const bool bvh_ok = build_segments(s->prims, bvh_segs, bvh_nodes, bvh_order, force_bvh, &bvh_extent);
  if (!bvh_ok) {
    bvh_segs.clear();
    bvh_nodes.clear();
    bvh_order.clear();
  }
  size_t off = 0;
  c->off_mat = off;
  off = align_up(off + m * 16, 256);
  c->off_cls = off;
  off = align_up(off + m * 4, 256);
  c->off_att = off;
  off = align_up(off + (static_cast<size_t>(n) + 1) * 16, 256);  // + the unit entry
  c->off_rec = off;
  off = align_up(off + m * 64, 256);
  c->off_bvh = off;
  off = align_up(off + (bvh_nodes.size() ? bvh_nodes.size() : 1) * sizeof(BvhNode), 256);
  c->off_bvh_order = off;
  off = align_up(off + (bvh_order.size() ? bvh_order.size() : 1) * 4, 256);
  c->off_lrec = off;
  off = align_up(off + (bvh_order.size() ? bvh_order.size() : 1) * 64, 256);
  c->off_segs = off;
  off = align_up(off + (bvh_segs.size() ? bvh_segs.size() : 1) * sizeof(BvhSegment), 256);
  // kind runs: maximal runs of consecutive primitives of one kind, in list order
  std::vector<uint32_t> runs;
  for (uint32_t i = 0; i < n;) {
    const uint32_t k = s->prims[i].kind <= FR_TRIANGLE ? s->prims[i].kind : FR_STUB;
    uint32_t j = i + 1;
    while (j < n && (s->prims[j].kind <= FR_TRIANGLE ? s->prims[j].kind : FR_STUB) == k) ++j;
    runs.insert(runs.end(), {k, i, j, 0u});
    i = j;
  }
  c->n_runs = static_cast<uint32_t>(runs.size() / 4);
  c->off_runs = off;
  off = align_up(off + (runs.size() ? runs.size() : 4) * 4, 256);
  c->off_acls = off;
  off = align_up(off + m * 4, 256);
  c->off_acls_att = off;
  off = align_up(off + (kNibbleMaxPrims + 1) * 16, 256);
  std::vector<unsigned char> host(off, 0);
  std::vector<float4> aclass;  // distinct attenuations, first appearance order
  bool aclass_ok = true;
  bool nonneg = true;
  bool diffuse = true;
  if (!bvh_nodes.empty()) memcpy(&host[c->off_bvh], bvh_nodes.data(), bvh_nodes.size() * sizeof(BvhNode));
  if (!bvh_order.empty()) memcpy(&host[c->off_bvh_order], bvh_order.data(), bvh_order.size() * 4);
  if (!bvh_segs.empty()) memcpy(&host[c->off_segs], bvh_segs.data(), bvh_segs.size() * sizeof(BvhSegment));
  if (!runs.empty()) memcpy(&host[c->off_runs], runs.data(), runs.size() * 4);
  c->bvh_ok = bvh_ok;
  c->bvh_extent = bvh_extent;
  c->n_segs = static_cast<uint32_t>(bvh_segs.size());
  c->bvh_levels = bvh_ok ? std::min(bvh_max_depth(bvh_segs, bvh_nodes) + 1u, kBvhStack) : kBvhStack;
  for (uint32_t i = 0; i < n; ++i) {
    const fr_prim& p = s->prims[i];
    uint32_t kind = p.kind;
    float4 g[4] = {};
    switch (p.kind) {
      case FR_SPHERE: g[0] = make_float4(p.g[0], p.g[1], p.g[2], p.g[3]); break;
      case FR_AABB:
        g[0] = make_float4(p.g[0], p.g[1], p.g[2], 0.0f);
        g[1] = make_float4(p.g[3], p.g[4], p.g[5], 0.0f);
        break;
      case FR_PLANE:
        g[0] = make_float4(p.g[0], p.g[1], p.g[2], 0.0f);
        g[1] = make_float4(p.g[3], p.g[4], p.g[5], 0.0f);
        g[2] = make_float4(p.g[6], p.g[7], p.g[8], 0.0f);
        break;
      case FR_OBB:
        g[0] = make_float4(p.g[0], p.g[1], p.g[2], p.g[12]);
        g[1] = make_float4(p.g[3], p.g[4], p.g[5], p.g[13]);
        g[2] = make_float4(p.g[6], p.g[7], p.g[8], p.g[14]);
        g[3] = make_float4(p.g[9], p.g[10], p.g[11], 0.0f);
        break;
      case FR_TRIANGLE: {
        // v0, edges e1 = v1 - v0 and e2 = v2 - v0, and the unit winding normal
        // unit(cross(e1, e2)), all in host f32 exactly as the oracle forms them
        const V3 v0{p.g[0], p.g[1], p.g[2]};
        const V3 e1 = sub(V3{p.g[3], p.g[4], p.g[5]}, v0), e2 = sub(V3{p.g[6], p.g[7], p.g[8]}, v0);
        const V3 nw = unit(cross(e1, e2));
        g[0] = make_float4(v0.x, v0.y, v0.z, 0.0f);
        g[1] = make_float4(e1.x, e1.y, e1.z, 0.0f);
        g[2] = make_float4(e2.x, e2.y, e2.z, 0.0f);
        g[3] = make_float4(nw.x, nw.y, nw.z, 0.0f);
        break;
      }
      default: kind = FR_STUB;
    }
    const uint32_t cls = scatter_class(p);
    if (cls == SC_METAL || cls == SC_DIELECTRIC) diffuse = false;
    const float4 mat = make_float4(p.color[0], p.color[1], p.color[2], p.fuzz);
    const float4 att = cls == SC_LIGHT ? make_float4(1.0f, 1.0f, 1.0f, 0.0f)
                                       : make_float4(p.color[0], p.color[1], p.color[2], 0.0f);
    memcpy(&host[c->off_mat + 16 * i], &mat, 16);
    memcpy(&host[c->off_cls + 4 * i], &cls, 4);
    memcpy(&host[c->off_att + 16 * i], &att, 16);
    {
      uint32_t k = 0;
      while (k < aclass.size() && memcmp(&aclass[k], &att, 12) != 0) ++k;
      if (k == aclass.size()) {
        if (aclass.size() < kNibbleMaxPrims)
          aclass.push_back(att);
        else
          aclass_ok = false;
      }
      const uint32_t kc = k < kNibbleMaxPrims ? k : 0u;
      memcpy(&host[c->off_acls + 4 * i], &kc, 4);
    }
    for (float a : {att.x, att.y, att.z})
      if (!(a >= 0.0f) || std::signbit(a) || !std::isfinite(a)) nonneg = false;
    memcpy(&g[3].w, &kind, 4);  // kind bits in g3.w
    memcpy(&host[c->off_rec + 64 * i], g, 64);
  }
  c->rec_words.resize(16u * static_cast<size_t>(n));
  if (n) memcpy(c->rec_words.data(), &host[c->off_rec], 64u * static_cast<size_t>(n));
  c->att_nonneg = nonneg;
  c->diffuse = diffuse;
  c->n_aclass = aclass_ok && n ? static_cast<uint32_t>(aclass.size()) : 0u;
  for (uint32_t k = 0; k <= kNibbleMaxPrims; ++k) {  // entries past the classes: the unit attenuation
    const float4 a = k < aclass.size() ? aclass[k] : make_float4(1.0f, 1.0f, 1.0f, 0.0f);
    memcpy(&host[c->off_acls_att + 16 * k], &a, 16);
  }
  // the BVH leaves' records, in leaf-slot order; a sphere's carries RN(radius^2) in place of
  // its radius, the product its hit test forms (sphere.rs:34; one VALU per leaf test saved)
  for (size_t slot = 0; slot < bvh_order.size(); ++slot) {
    float* lr = reinterpret_cast<float*>(&host[c->off_lrec + 64 * slot]);
    memcpy(lr, &host[c->off_rec + 64 * static_cast<size_t>(bvh_order[slot])], 64);
    uint32_t kind;
    memcpy(&kind, &lr[15], 4);
    if (kind == FR_SPHERE) lr[3] = lr[3] * lr[3];
  }
  {
    // entry n: the unit attenuation the depth-8 stack's empty levels point at
    const float4 one = make_float4(1.0f, 1.0f, 1.0f, 0.0f);
    memcpy(&host[c->off_att + 16 * n], &one, 16);
  }
  if (n == 0) {
    const uint32_t stub = FR_STUB;
    memcpy(&host[c->off_rec + 60], &stub, 4);
  }
  HIPCHK(hipMalloc(&c->blob, off));
  HIPCHK(hipMemcpy(c->blob, host.data(), off, hipMemcpyHostToDevice));
  c->n = n;
  c->has_plane = false;
  c->kinds = 0;
  for (const fr_prim& p : s->prims) {
    c->has_plane |= p.kind == FR_PLANE;
    c->kinds |= 1u << (p.kind <= FR_TRIANGLE ? p.kind : FR_STUB);
  }
  c->version = s->version;
  static std::atomic<uint64_t> g_uploads{0};
  c->uid = ++g_uploads;
  *out = c;
  return FR_OK;
}

void release_device_copies(fr_scene* s) {
  std::lock_guard<std::mutex> g(s->mu);
  for (DeviceCopy* c : s->copies) {
    if (c->blob) {
      int cur = 0;
      if (hipGetDevice(&cur) == hipSuccess) {
        (void)hipSetDevice(c->device);
        (void)hipFree(c->blob);
        (void)hipSetDevice(cur);
      }
    }
    delete c;
  }
  s->copies.clear();
}

}  // namespace fr

using namespace fr;

constexpr int kCntWords = 64;  // counter words per frame slot (fr_ctx::d_cnt)

struct fr_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  hipEvent_t ev0 = nullptr, ev1 = nullptr, ev_start = nullptr;
  std::vector<hipEvent_t> ev_trace;  // start/stop pairs around each pass's trace kernel
  std::vector<hipEvent_t> ev_sum;    // end of each pass's sum kernel
  // Pass pipeline: traces alternate between `stream` and `stream2`,
  // sums run on `stream_sum`, so a pass's sum and tail overlap the next pass's trace.
  hipStream_t stream2 = nullptr, stream_sum = nullptr;
  // fr_ctx_download_async: D2H copies of the last render on their own stream; the next
  // render's first sum kernel (the first writer of d_mean / d_u8) waits for ev_copy, so a
  // frame's gather overlaps the next frame's trace.
  hipStream_t stream_copy = nullptr;
  hipEvent_t ev_copy = nullptr;
  bool copy_pending = false;
  int passes = 0;
  int occupancy = 0;  // trace-kernel workgroups per CU of the last launch (occupancy API)
  float* d_mean = nullptr;
  uint8_t* d_u8 = nullptr;
  // [0..3] counters, [4..30] and [32..63] diagnostics (FR_SECCNT, FR_PROF, FR_DIAG builds);
  // [31] queue head: one set of kCntWords per frame slot
  unsigned long long* d_cnt = nullptr;
  unsigned long long* last_cnt = nullptr;  // the last render's set
  // Frame pipeline (FR_FRAME_PIPE): one-pass frames alternate between two
  // frame slots (sample buffer half, counter set), so frame k+1's trace starts when frame k's
  // trace ends while frame k's sum runs beside it; ev_fslot[s] = the end of the last sum
  // that used slot s, which the next frame on that slot waits for.
  static constexpr int kFrameSlots = 4;  // at most (FR_FRAME_SLOTS, default 2)
  int frame_slot = 0, frame_parity = 0;
  int fs_n = 0;            // slots in the current layout (2 to 4; 0: not pipelined)
  size_t fs_bytes = 0;     // sample-buffer bytes per slot in that layout
  hipEvent_t ev_fslot[kFrameSlots] = {};
  bool fslot_used[kFrameSlots] = {};
  unsigned long long* d_wcnt = nullptr;  // per-wave partial counters (KWork::wave_counters)
  uint32_t wcnt_waves = 0;               // their capacity in waves
  float* d_samples = nullptr;
  float* d_running = nullptr;
  size_t cap_pixels = 0, cap_samples = 0, cap_running = 0;
  int num_cus = 0;
  size_t device_bytes = 0;  // HBM size (the sample buffer budget's default)
  fr_params last{};
  uint32_t last_n = 0;
  bool pending = false;
  // the last render was enqueued while the one before it still ran (frames streamed): the
  // next render reserves slots for overlapping even if it finds the device idle (render_ctx)
  bool streaming = false;
  std::chrono::steady_clock::time_point t0;
  // fr_ctx_trace_log: event pairs around every trace launch since the log was enabled,
  // across renders (ev_trace holds only the last render's), so a caller streaming K
  // frames can average the kernel's duration over all of them
  // log 0: trace launches (on the launch's stream); log 1: whole renders (ev0 .. ev1)
  // the last render's trace kernel: scene-specialised (jit.h) or compiled in
  bool jit_used = false;
  JitStats jit_stats{};
  int jit_state = FR_JIT_OFF;
  // the scene kernel the last lookup found and what it was for (upload, specialisation
  // flags), pinned loaded: a frame of the same scene and shape skips the lookup (its
  // prelude and key hashing are ~0.1 ms of host time per render)
  hipFunction_t jc_fn = nullptr;
  std::shared_ptr<void> jc_pin;
  uint64_t jc_uid = 0;
  uint32_t jc_flags = 0;
  bool jc_small = false;
  bool log_on = false;
  std::vector<hipEvent_t> log_ev[2];  // 2 per entry (start, end); reused across logs
  size_t log_n[2] = {0, 0};           // entries logged
};

static hipError_t log_event(fr_ctx* c, int which, size_t k, hipStream_t st) {
  std::vector<hipEvent_t>& v = c->log_ev[which];
  while (v.size() <= k) {
    hipEvent_t e;
    const hipError_t err = hipEventCreate(&e);
    if (err != hipSuccess) return err;
    v.push_back(e);
  }
  return hipEventRecord(v[k], st);
}
static hipError_t log_start(fr_ctx* c, int which, hipStream_t st) {
  return log_event(c, which, 2 * c->log_n[which], st);
}
static hipError_t log_end(fr_ctx* c, int which, hipStream_t st) {
  const hipError_t e = log_event(c, which, 2 * c->log_n[which] + 1, st);
  if (e == hipSuccess) ++c->log_n[which];
  return e;
}

// Picks the specialisation: single-kind scenes (all boxes, all spheres) drop the
// per-primitive kind switch; HAS_PLANE adds the stale-record bookkeeping; small depth
// uses the u16 stack with the unrolled unwind.
// Persistent grid: as many workgroups as are resident at once (the occupancy API reads the
// kernel's registers and this launch's LDS), or fewer for a small pass. A workgroup
// beyond the resident count would start only after the queue has drained.
struct Grid {
  uint64_t want;  // workgroups the pass could use (items / kBlock)
  int num_cus;
  int* per_cu;    // out: resident workgroups per CU
  uint32_t* blocks;  // out: workgroups launched
  size_t stage_bytes;  // BVH kernels: LDS for sample staging, taken if it costs no residency
  uint32_t reserve = 0;  // workgroup slots per CU left free (frame pipeline: the previous frame's sum)
};

// The scene-specialised kernel request of one render (jit.h): on for list-loop launches
// when the caller asks (FR_FLAG_SCENE_JIT or FR_SCENE_JIT=1) and the scene is small.
struct JitReq {
  bool on = false;
  bool wait = false;  // compile on this thread if needed (fr_ctx_prepare, FR_FLAG_SCENE_JIT_WAIT)
  bool cached_only = false;  // FR_FLAG_SCENE_JIT_CACHED: never compile or queue (one-shot callers)
  std::shared_ptr<void> pin;  // the scene kernel's module: its launches are noted (jit_note_launch)
  int device = 0;
  const DeviceCopy* dc = nullptr;
  bool dry = false;   // fr_ctx_prepare: get the kernel, launch nothing
  bool resolved = false;     // the lookup ran (once per render: the dry pre-step)
  hipFunction_t fn = nullptr;  // its result: the scene kernel, or null (compiled-in kernel)
  bool used = false;  // out: the launch ran the scene-specialised kernel
  JitStats stats{};   // out: the lookup's time and state
};

// The host build's tuning and contract macros, so the run-time build of trace_kernel.h
// is the same specialisation as the one compiled into the library, with only the list
// walk replaced.
static std::string jit_defines() {
  std::string d;
  auto def = [&](const char* name, long v) { d += std::string("#define ") + name + " " + std::to_string(v) + "\n"; };
  def("FR_KREJ", FR_KREJ);
  def("FR_KREJ_NIB", FR_KREJ_NIB);
  def("FR_CLAIM_MIN", FR_CLAIM_MIN);
  def("FR_CLAIM_MIN_NIB", FR_CLAIM_MIN_NIB);
  def("FR_NUM_SGPR", FR_NUM_SGPR);
  def("FR_BLOCK_SAMPLES", FR_BLOCK_SAMPLES);
  def("FR_FINE_SAMPLES", FR_FINE_SAMPLES);
  def("FR_STAGE", FR_STAGE);
  def("FR_BVH_STAGE", FR_BVH_STAGE);
  def("FR_STAGE_SMAJOR", FR_STAGE_SMAJOR);
#ifdef FR_TRACE_PRIO
  def("FR_TRACE_PRIO", FR_TRACE_PRIO);
#endif
#ifdef FR_SKY_DEFER
  d += "#define FR_SKY_DEFER\n";
#endif
#ifdef FR_MIN_WAVES
  def("FR_MIN_WAVES", FR_MIN_WAVES);
#else
  def("FR_NIB_WAVES", FR_NIB_WAVES);
  def("FR_DIFF12_WAVES", FR_DIFF12_WAVES);
#endif
#ifdef FR_CAM_RESIDENT
  d += "#define FR_CAM_RESIDENT\n";
#endif
#ifdef FR_SPHERE_IEEE
  d += "#define FR_SPHERE_IEEE\n";
#endif
#ifdef FR_SKY_IEEE
  d += "#define FR_SKY_IEEE\n";
#endif
#ifdef FR_DIV_2STEP
  d += "#define FR_DIV_2STEP\n";
#endif
#ifdef FR_NO_UNROLL_NIB
  d += "#define FR_NO_UNROLL_NIB\n";
#endif
#if FR_BOX_FMA
  def("FR_BOX_FMA", FR_BOX_FMA);
#endif
#ifdef FR_PROF
  d += "#define FR_PROF\n";  // section clocks go to the launch's counters, not device globals
#endif
#ifdef FR_SECCNT
  d += "#define FR_SECCNT\n";  // region entry counts go to the launch's counters (tools/isa_sections.py)
#endif
  return d;
}

template <int KS, bool HP, int KREJ, int MAXD, bool BV, bool MT, int DEFER, int MAT = 0>
static int launch_persistent(const Grid& g, size_t lds, hipStream_t st, KArgs a, JitReq* jr) {
  auto kern = trace_kernel<KS, HP, KREJ, MAXD, BV, MT, DEFER, MAT>;
  hipFunction_t jfn = nullptr;
  if (!BV && jr && jr->on) {
    if (!jr->resolved) {
      char name[160];
      snprintf(name, sizeof name, "fr::trace_kernel<%d, %s, %d, %d, %s, %s, %d, %d>", KS, HP ? "true" : "false", KREJ,
               MAXD, BV ? "true" : "false", MT ? "true" : "false", DEFER, MAT);
      const int targs[8] = {KS, HP, KREJ, MAXD, BV, MT, DEFER, MAT};
      const bool tbool[8] = {false, true, false, false, true, true, false, false};
      const JitSpec spec{name, targs, tbool, 8, jit_defines(), jr->dc->rec_words.data(), jr->dc->n};
      const int rc = jit_trace_kernel(jr->device, spec, jr->wait, &jr->fn, &jr->stats, jr->cached_only);
      if (rc) return rc;
      jr->resolved = true;
    }
    jfn = jr->fn;  // null while the compile is pending (or failed): the compiled-in kernel runs
    jr->used = jfn != nullptr;
  }
  if (jr && jr->dry) return FR_OK;
  int per_cu = 0;
  const hipError_t oe =
      jfn ? hipModuleOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, jfn, static_cast<int>(kBlock), lds)
          : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, static_cast<int>(kBlock), lds);
  if (oe != hipSuccess || per_cu < 1) per_cu = 1;
  // the per-wave counter slots (fr_ctx::d_wcnt) hold kMaxWgPerCu workgroups per CU
  if (per_cu > static_cast<int>(kMaxWgPerCu)) per_cu = static_cast<int>(kMaxWgPerCu);
  // BVH kernels store their samples unstaged unless FR_BVH_STAGE asks: "1" staged even at a
  // lower residency, "2" staged when it costs no residency (A/B, tests). At 7 workgroups per
  // CU the pair staging measured slower than plain stores (C5 51.45 ms unstaged, 51.87
  // staged; with 8-bin trees 48.39 / 48.63); at 6 it had paid (66.8 -> 64.3 ms, round 2).
  const char* stage_env = getenv("FR_BVH_STAGE");
  const bool force_stage = stage_env && strcmp(stage_env, "1") == 0;
  if (g.stage_bytes && stage_env && (force_stage || strcmp(stage_env, "2") == 0)) {
    int staged = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&staged, kern, static_cast<int>(kBlock), lds + g.stage_bytes) ==
            hipSuccess &&
        (staged >= per_cu || (force_stage && staged >= 1))) {
      per_cu = staged < static_cast<int>(kMaxWgPerCu) ? staged : static_cast<int>(kMaxWgPerCu);
      lds += g.stage_bytes;
      a.kp.flags |= KF_STAGE;
    }
  }
  // only full 8-workgroup grids give a slot up: the BVH kernels (6 per CU) lost a sixth of
  // their grid for a sum of a twentieth of their frame (C5 55.6 -> 58.0 ms)
  if (g.reserve && per_cu >= static_cast<int>(kMaxWgPerCu)) per_cu -= static_cast<int>(g.reserve);
  *g.per_cu = per_cu;
  uint64_t cap = static_cast<uint64_t>(per_cu) * static_cast<uint64_t>(g.num_cus);
  // FR_MAX_WGS=k caps the grid (tests: with a few workgroups every wave claims many
  // batches, partly used ones included, so the claim paths run at small image sizes)
  if (const char* e = getenv("FR_MAX_WGS"))
    if (atoi(e) > 0 && static_cast<uint64_t>(atoi(e)) < cap) cap = static_cast<uint64_t>(atoi(e));
  const uint32_t blocks = static_cast<uint32_t>(g.want < cap ? (g.want ? g.want : 1u) : cap);
  *g.blocks = blocks;
  a.kp.n_static = blocks * kBlock;  // one 64-item batch per wave of the grid
  if (jfn) {
    // the same by-value KArgs at kernarg offset 0 as the compiled-in kernels take
    size_t bytes = sizeof(KArgs);
    void* cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, &a, HIP_LAUNCH_PARAM_BUFFER_SIZE, &bytes, HIP_LAUNCH_PARAM_END};
    HIPCHK(hipModuleLaunchKernel(jfn, blocks, 1, 1, kBlock, 1, 1, static_cast<uint32_t>(lds), st, nullptr, cfg));
    jit_note_launch(jr->pin, st);  // an LRU eviction waits for the last launch on every stream used
  } else {
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(kBlock), lds, st, a);
  }
  return FR_OK;
}

template <int KS, bool HP, bool BV, bool MT = false>
static int launch_depth(bool small_depth, const Grid& g, size_t lds, hipStream_t st, const KArgs& a, JitReq* jr) {
  if constexpr (BV && !MT) {
    // diffuse scenes of <= 15 distinct attenuations: 8-B records of attenuation classes
    if ((a.kp.flags & KF_DEFER) && (a.kp.flags & KF_NIBBLE) && (a.kp.flags & KF_DIFFUSE))
      return launch_persistent<KS, HP, FR_KREJ_BVH, kSmallDepth, true, false, 2, 1>(g, lds, st, a, jr);
  }
  if constexpr (!BV && !MT) {
    if (a.kp.flags & KF_DEFER) {
      if ((a.kp.flags & KF_NIBBLE) && (a.kp.flags & KF_DIFFUSE))
        return launch_persistent<KS, HP, FR_KREJ_NIB, kSmallDepth, false, false, 2, 1>(g, lds, st, a, jr);
      if (a.kp.flags & KF_NIBBLE)
        return launch_persistent<KS, HP, FR_KREJ_NIB, kSmallDepth, false, false, 2>(g, lds, st, a, jr);
      if (a.kp.flags & KF_DIFFUSE)
        return launch_persistent<KS, HP, FR_KREJ, kSmallDepth, false, false, 1, 1>(g, lds, st, a, jr);
      return launch_persistent<KS, HP, FR_KREJ, kSmallDepth, false, false, 1>(g, lds, st, a, jr);
    }
  }
  const bool diffuse = (a.kp.flags & KF_DIFFUSE) != 0;
  if (small_depth && diffuse) return launch_persistent<KS, HP, FR_KREJ, kSmallDepth, BV, MT, 0, 1>(g, lds, st, a, jr);
  if (small_depth) return launch_persistent<KS, HP, FR_KREJ, kSmallDepth, BV, MT, 0>(g, lds, st, a, jr);
  if (diffuse) return launch_persistent<KS, HP, FR_KREJ, 0, BV, MT, 0, 1>(g, lds, st, a, jr);
  return launch_persistent<KS, HP, FR_KREJ, 0, BV, MT, 0>(g, lds, st, a, jr);
}

// BVH kernels walk the list's segments (bvh.h); scenes with planes use the general
// kernel, which tests each plane in list order between the runs.
static int launch_trace(uint32_t kinds, bool has_plane, bool bvh, bool small_depth, const Grid& g, size_t lds,
                        hipStream_t st, const KArgs& a, JitReq* jr) {
  if (a.kp.flags & FR_FLAG_MT_BANDS) {  // save_image_mt: the general kernels, in-order loop
    if (has_plane) return launch_depth<KS_ANY, true, false, true>(small_depth, g, lds, st, a, jr);
    return launch_depth<KS_ANY, false, false, true>(small_depth, g, lds, st, a, jr);
  }
  if (kinds == (1u << FR_AABB)) {
    if (bvh) return launch_depth<KS_AABB, false, true>(small_depth, g, lds, st, a, jr);
    return launch_depth<KS_AABB, false, false>(small_depth, g, lds, st, a, jr);
  }
  if (kinds == (1u << FR_SPHERE)) {
    if (bvh) return launch_depth<KS_SPHERE, false, true>(small_depth, g, lds, st, a, jr);
    return launch_depth<KS_SPHERE, false, false>(small_depth, g, lds, st, a, jr);
  }
  if (has_plane) {
    if (bvh) return launch_depth<KS_ANY, true, true>(small_depth, g, lds, st, a, jr);
    return launch_depth<KS_ANY, true, false>(small_depth, g, lds, st, a, jr);
  }
  if (bvh) return launch_depth<KS_ANY, false, true>(small_depth, g, lds, st, a, jr);
  return launch_depth<KS_ANY, false, false>(small_depth, g, lds, st, a, jr);
}

// Bytes of per-sample colours one pass may hold (FR_SAMPLE_BUFFER_GB, default 8).
// Sample buffer budget: FR_SAMPLE_BUFFER_GB, else min(32 GiB, 1/8 of the device's HBM)
// (32 GiB on MI355X: C4's shard and C5 trace in one pass)
static size_t sample_buffer_cap(size_t device_bytes) {
  double gb = device_bytes ? static_cast<double>(device_bytes) / 8.0 / (1ull << 30) : 8.0;
  if (gb > 32.0) gb = 32.0;
  if (const char* e = getenv("FR_SAMPLE_BUFFER_GB")) gb = atof(e);
  if (gb < 0.001) gb = 0.001;
  return static_cast<size_t>(gb * (1ull << 30));
}

static int check_params(const fr_params* p) {
  if (!p) return set_error(FR_EARG, "null params");
  if (p->width == 0 || p->height == 0) return set_error(FR_EARG, "width/height must be > 0");
  if (static_cast<uint64_t>(p->width) * p->height > (1ull << 31))
    return set_error(FR_EARG, "image too large (pixel index must fit in 31 bits)");
  if (p->width > 65535 || p->height > 65535)
    return set_error(FR_EARG, "width/height must be < 65536 (packed pixel coordinates)");
  if (p->max_depth > kMaxDepth) return set_error(FR_EARG, "max_depth %u > %u", p->max_depth, kMaxDepth);
  if (p->strip_rows != kStripRows) return set_error(FR_EARG, "strip_rows must be %u", kStripRows);
  if (p->shard_count == 0 || p->shard_index >= p->shard_count)
    return set_error(FR_EARG, "shard_index %u / shard_count %u invalid", p->shard_index, p->shard_count);
  return FR_OK;
}

extern "C" {

int fr_device_count(int* count) {
  if (!count) return set_error(FR_EARG, "null count");
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return set_error(FR_ENODEV, "hipGetDeviceCount: %s", hipGetErrorString(e));
  }
  *count = n;
  return FR_OK;
}

int fr_ctx_create(int device, void* stream, fr_ctx** out) {
  if (!out) return set_error(FR_EARG, "fr_ctx_create: null output");
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return set_error(FR_ENODEV, "no HIP device");
  if (device < 0 || device >= n) return set_error(FR_ENODEV, "device %d not present (%d devices)", device, n);
  SET_DEVICE(device);
  fr_ctx* c = new fr_ctx();
  c->device = device;
  if (stream) {
    c->stream = static_cast<hipStream_t>(stream);
  } else {
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
      delete c;
      return set_error(FR_EHIP, "hipStreamCreate failed");
    }
    c->own_stream = true;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) {
    c->num_cus = prop.multiProcessorCount;
    c->device_bytes = prop.totalGlobalMem;
  }
  if (c->num_cus <= 0) c->num_cus = 256;
  if (hipEventCreate(&c->ev0) != hipSuccess || hipEventCreate(&c->ev1) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_start, hipEventDisableTiming) != hipSuccess ||
      hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->stream_sum, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&c->stream_copy, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_copy, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fslot[0], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fslot[1], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fslot[2], hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&c->ev_fslot[3], hipEventDisableTiming) != hipSuccess ||
      hipMalloc(&c->d_cnt, fr_ctx::kFrameSlots * kCntWords * sizeof(unsigned long long)) != hipSuccess ||
      hipMalloc(&c->d_wcnt, fr_ctx::kFrameSlots * 3 * sizeof(unsigned long long) * kMaxWgPerCu * (kBlock / 64u) *
                                c->num_cus) !=
          hipSuccess) {  // one set per pass slot (traces of consecutive passes overlap)
    fr_ctx_free(c);
    return set_error(FR_EHIP, "fr_ctx_create: event/counter allocation failed");
  }
  *out = c;
  return FR_OK;
}

void fr_ctx_free(fr_ctx* c) {
  if (!c) return;
  int cur = -1;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(c->device);
  // every stream drained before any buffer or event it may still use goes
  for (hipStream_t s : {c->stream, c->stream2, c->stream_sum, c->stream_copy})
    if (s) (void)hipStreamSynchronize(s);
  if (c->stream_copy) (void)hipStreamSynchronize(c->stream_copy), (void)hipStreamDestroy(c->stream_copy);
  if (c->ev_copy) (void)hipEventDestroy(c->ev_copy);
  for (hipEvent_t e : c->ev_fslot)
    if (e) (void)hipEventDestroy(e);
  if (c->d_mean) (void)hipFree(c->d_mean);
  if (c->d_u8) (void)hipFree(c->d_u8);
  if (c->d_cnt) (void)hipFree(c->d_cnt);
  if (c->d_wcnt) (void)hipFree(c->d_wcnt);
  if (c->d_samples) (void)hipFree(c->d_samples);
  if (c->d_running) (void)hipFree(c->d_running);
  for (hipEvent_t e : c->ev_trace) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->ev_sum) (void)hipEventDestroy(e);
  for (auto& v : c->log_ev)
    for (hipEvent_t e : v) (void)hipEventDestroy(e);
  if (c->ev_start) (void)hipEventDestroy(c->ev_start);
  if (c->stream2) (void)hipStreamSynchronize(c->stream2), (void)hipStreamDestroy(c->stream2);
  if (c->stream_sum) (void)hipStreamSynchronize(c->stream_sum), (void)hipStreamDestroy(c->stream_sum);
  if (c->ev0) (void)hipEventDestroy(c->ev0);
  if (c->ev1) (void)hipEventDestroy(c->ev1);
  if (c->own_stream && c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  if (cur >= 0) (void)hipSetDevice(cur);  // the caller's current device (torch's) stays as it was
}

static int render_impl(fr_ctx* c, fr_scene* scene, const fr_camera* cam, const fr_params* p, bool dry);

int fr_ctx_render(fr_ctx* c, fr_scene* scene, const fr_camera* cam, const fr_params* p) {
  return render_impl(c, scene, cam, p, false);
}

int fr_ctx_prepare(fr_ctx* c, fr_scene* scene, const fr_camera* cam, const fr_params* p) {
  return render_impl(c, scene, cam, p, true);
}

// dry (fr_ctx_prepare): everything a render of these parameters sets up before its first
// launch — the scene's device copy, the output and sample buffers, the scene-specialised
// kernel when asked for — and nothing enqueued.
static int render_impl(fr_ctx* c, fr_scene* scene, const fr_camera* cam, const fr_params* p, bool dry) {
  if (!c || !scene || !cam) return set_error(FR_EARG, "fr_ctx_render: null argument");
  int rc = check_params(p);
  if (rc) return rc;
  SET_DEVICE(c->device);
  DeviceCopy* dc = nullptr;
  rc = upload_scene(scene, c->device, &dc);
  if (rc) return rc;
  const size_t pixels = static_cast<size_t>(p->width) * p->height;
  if (pixels > c->cap_pixels) {
    if (c->copy_pending) HIPCHK(hipStreamSynchronize(c->stream_copy));  // a gather still reads them
    if (c->d_mean) HIPCHK(hipFree(c->d_mean));
    if (c->d_u8) HIPCHK(hipFree(c->d_u8));
    c->d_mean = nullptr;
    c->d_u8 = nullptr;
    c->cap_pixels = 0;
    HIPCHK(hipMalloc(&c->d_mean, pixels * 3 * sizeof(float)));
    HIPCHK(hipMalloc(&c->d_u8, pixels * 3));
    c->cap_pixels = pixels;
  }
  KScene ks;
  const char* b = static_cast<const char*>(dc->blob);
  ks.rec = reinterpret_cast<const float4*>(b + dc->off_rec);
  ks.mat = reinterpret_cast<const float4*>(b + dc->off_mat);
  ks.cls = reinterpret_cast<const uint32_t*>(b + dc->off_cls);
  ks.att = reinterpret_cast<const float4*>(b + dc->off_att);
  ks.acls = reinterpret_cast<const uint32_t*>(b + dc->off_acls);
  ks.n = dc->n;
  // FR_BVH=0 forces the in-order loop (A/B and tests)
  const char* bvh_env = getenv("FR_BVH");
  // the node cull holds for origins within kBvhOriginReach scene extents (bvh.h)
  const float cam_reach = std::max(std::max(fabsf(cam->position[0]), fabsf(cam->position[1])),
                                   fabsf(cam->position[2])) + fabsf(cam->lens_radius);
  const bool cam_near = cam_reach <= kBvhOriginReach * (dc->bvh_extent + 1.0f);
  // save_image_mt renders run the in-order list kernels (launch_trace), whose LDS layout
  // (sample staging, no traversal stack) the size below must follow
  const bool use_bvh = dc->bvh_ok && dc->n_segs > 0 && cam_near && !(bvh_env && strcmp(bvh_env, "0") == 0) &&
                       !(p->flags & FR_FLAG_MT_BANDS);
  ks.bvh = reinterpret_cast<const float4*>(b + dc->off_bvh);
  ks.bvh_order = reinterpret_cast<const uint32_t*>(b + dc->off_bvh_order);
  ks.lrec = reinterpret_cast<const float4*>(b + dc->off_lrec);
  ks.segs = reinterpret_cast<const uint4*>(b + dc->off_segs);
  ks.runs = reinterpret_cast<const uint4*>(b + dc->off_runs);
  ks.n_runs = dc->n_runs;
  ks.n_segs = use_bvh ? dc->n_segs : 0u;
  ks.reach = kBvhOriginReach * (dc->bvh_extent + 1.0f);
  ks.att_nonneg = dc->att_nonneg ? 1u : 0u;
  KCam kc;
  kc.px = cam->position[0], kc.py = cam->position[1], kc.pz = cam->position[2];
  kc.lx = cam->lower_left[0], kc.ly = cam->lower_left[1], kc.lz = cam->lower_left[2];
  kc.hx = cam->horizontal[0], kc.hy = cam->horizontal[1], kc.hz = cam->horizontal[2];
  kc.vx = cam->vertical[0], kc.vy = cam->vertical[1], kc.vz = cam->vertical[2];
  kc.ux = cam->u[0], kc.uy = cam->u[1], kc.uz = cam->u[2];
  kc.bx = cam->v[0], kc.by = cam->v[1], kc.bz = cam->v[2];
  kc.lens = cam->lens_radius;
  kc.lens_s = ldexpf(kc.lens, -23);
  kc.lens_pre = std::isfinite(kc.lens) && ldexpf(kc.lens_s, 23) == kc.lens ? 1u : 0u;
  KParams kp;
  kp.W = p->width;
  kp.H = p->height;
  kp.rW = 1.0f / (static_cast<float>(p->width) * 16777216.0f);  // = RN(1 / W) 2^-24
  kp.rH = 1.0f / (static_cast<float>(p->height) * 16777216.0f);
  kp.sW = static_cast<float>(p->width) * 16777216.0f;
  kp.sH = static_cast<float>(p->height) * 16777216.0f;
  kp.spp = p->spp;
  kp.max_depth = p->max_depth;
  kp.seed = p->seed;
  kp.shard_index = p->shard_index;
  kp.shard_count = p->shard_count;
  kp.flags = p->flags;
  kp.tiles_per_row = (p->width + 7u) / 8u;
  kp.band_h = p->height / 4u;
  const uint32_t strips = (p->height + kStripRows - 1) / kStripRows;
  const uint32_t my_strips =
      strips > p->shard_index ? (strips - p->shard_index + p->shard_count - 1) / p->shard_count : 0u;
  kp.n_tiles = my_strips * kp.tiles_per_row;
  kp.P = kp.n_tiles * 64u;
  fastdiv_magic(kp.n_tiles, kp.tiles_magic, kp.tiles_shift);
  fastdiv_magic(kp.tiles_per_row, kp.row_magic, kp.row_shift);
  const uint32_t nblocks = (p->spp + kBlockSamples - 1) / kBlockSamples;
  // Passes of nb_pass blocks each. With more than one pass the sample buffer holds two
  // pass slots (a pass traces into one while the previous pass's sum reads the other).
  // FR_PIPELINE (default 1) asks for at least that many passes; the buffer budget
  // (FR_SAMPLE_BUFFER_GB) may force more. Two pipelined passes measured 0.6 % faster
  // on C3, but overlapping launches blur each launch's own HIP-event time (DESIGN.md
  // §4.6), so one pass is the default.
  // sample slots per item: a frame of spp < 16 (update()'s 1-spp frames) needs only spp
  kp.ks = p->spp < kBlockSamples ? (p->spp ? p->spp : 1u) : kBlockSamples;
  const bool small_depth = p->max_depth <= kSmallDepth && dc->n < 65536u;
  // the deferred unwind (kDeferMaxPrims); FR_DEFER=0 keeps the unwind in the trace kernel,
  // FR_DEFER=1 the 12-B records for small scenes too (A/B)
  const char* defer_env = getenv("FR_DEFER");
  // FR_MAT=0 keeps the general shading step for diffuse-only scenes (A/B, tests)
  const char* mat_env = getenv("FR_MAT");
  const bool diffuse_k = dc->diffuse && !(mat_env && strcmp(mat_env, "0") == 0);
  // BVH kernels defer too when the scene is diffuse and has at most 15 distinct attenuations
  // (C5: one): 8-B records of attenuation classes
  const bool bvh_nib = use_bvh && small_depth && diffuse_k && dc->n_aclass > 0 &&
                       !(p->flags & FR_FLAG_MT_BANDS) && !(defer_env && strcmp(defer_env, "0") == 0);
  const bool defer = bvh_nib || (small_depth && dc->n <= kDeferMaxPrims && !use_bvh &&
                                 !(p->flags & FR_FLAG_MT_BANDS) && !(defer_env && strcmp(defer_env, "0") == 0));
  const bool nibble =
      bvh_nib || (defer && dc->n <= kNibbleMaxPrims && !(defer_env && strcmp(defer_env, "1") == 0));
  if (defer) kp.flags |= KF_DEFER;
  if (nibble) kp.flags |= KF_NIBBLE;
  if (diffuse_k) kp.flags |= KF_DIFFUSE;
  const uint32_t wps = nibble && !kSkyDefer ? 2u : 3u;  // words per sample in the buffer
  const size_t per_block = static_cast<size_t>(kp.P) * kp.ks * wps * sizeof(float);
  uint32_t want_passes = 1;
  if (const char* e = getenv("FR_PIPELINE")) want_passes = static_cast<uint32_t>(atoi(e) > 0 ? atoi(e) : 1);
  uint32_t passes_u = nblocks ? (want_passes < nblocks ? want_passes : nblocks) : 0u;
  uint32_t nb_pass = passes_u ? (nblocks + passes_u - 1) / passes_u : 0u;
  const size_t cap_blocks = per_block ? sample_buffer_cap(c->device_bytes) / per_block : nblocks;
  // 32-bit item indices. After the queue drains, every wave may still bump the counter
  // once per lane (each claim retires >= 1 lane): <= 8 blocks/CU x 4 waves x 64 x 64 on
  // 256 CUs = 2^25 past n_items, so keep 2^28 of headroom below 2^32.
  constexpr uint32_t kItemLimit = 0xFFFFFFFFu - (1u << 28);
  // The pass holding the last block runs its kFineSub sub-blocks as items: up to
  // (nb + kFineSub - 1) x P items.
  const uint32_t fine_extra = nblocks > 1 ? kFineSub - 1u : 0u;
  if (kp.P && kItemLimit / kp.P < 1u + fine_extra)
    return set_error(FR_EARG, "shard of %u pixel slots exceeds the 32-bit work-item range at spp %u; use more shards",
                     kp.P, p->spp);
  uint32_t nb_max = static_cast<uint32_t>(passes_u > 1 ? cap_blocks / 2 : cap_blocks);
  if (kp.P && nb_max > kItemLimit / kp.P - fine_extra) nb_max = kItemLimit / kp.P - fine_extra;
  if (nb_max < 1) nb_max = 1;
  if (nb_pass > nb_max) {
    nb_pass = nb_max;
    if (nblocks > nb_pass && nb_pass > static_cast<uint32_t>(cap_blocks / 2) && cap_blocks / 2 >= 1)
      nb_pass = static_cast<uint32_t>(cap_blocks / 2);  // two slots must fit
  }
  const int passes = nb_pass ? static_cast<int>((nblocks + nb_pass - 1) / nb_pass) : 0;
  // frame pipeline (fr_ctx::frame_slot): one-pass frames whose sample buffer fits twice
  // (FR_FRAME_PIPE=0 turns it off). Streamed scene_08 frames, shard 0 of N on one MI355X:
  // 17.01 -> 16.59 ms at N = 1, 2.52 -> 2.29 ms at N = 8
  // Traces: frame k+1's trace follows frame k's on one stream, or, for a shard with fewer
  // than two pixel slots per grid lane (two items per lane and block or fewer: the queue's
  // drain is a large part of the frame, shards 0 of 4 and of 8), consecutive frames' traces
  // alternate between two streams, so the next frame's trace fills the CUs the previous
  // one's drain leaves idle: shard 0/8 2.47 -> 2.29 ms per frame, 0/4 4.27-4.46 -> 4.28
  // (steadier), the same at N = 1 and 2, where serial traces keep each launch's own event
  // time. FR_FRAME_PIPE=1 / 2 forces serial / overlapping traces.
  // Two slots (FR_FRAME_SLOTS=3 or 4 asks for more when the budget holds them). With round
  // 3's sum, which ran longer than the trace beside it, three slots let frame k + 2's trace
  // start before frame k's sum ended; since round 4's sum keeps pace, two are faster (C3
  // streamed 16.27 -> 16.17 ms per frame, N = 2 shards -0.3 %, N = 4 and 8 the same).
  const char* fp_env = getenv("FR_FRAME_PIPE");
  int want_fs = 2;
  if (const char* e = getenv("FR_FRAME_SLOTS"))
    want_fs = std::max(2, std::min(fr_ctx::kFrameSlots, atoi(e)));
  int nfs = 0;
  if (passes == 1 && !(fp_env && strcmp(fp_env, "0") == 0))
    for (int k = want_fs; k >= 2 && !nfs; --k)
      if (cap_blocks >= static_cast<uint64_t>(k) * nblocks) nfs = k;
  const bool fpipe = nfs > 0;
  const uint64_t grid_lanes = static_cast<uint64_t>(c->num_cus) * (kMaxWgPerCu - 1u) * kBlock;
  // (round 6: below three slots per grid lane, so N = 2 shards of a 1080p frame overlap too;
  // at N = 1 a launch's own HIP-event time stays the launch's, and the gain measured 0.3 %)
  const bool fpipe_overlap =
      fpipe && (fp_env && *fp_env ? strcmp(fp_env, "2") == 0 : static_cast<uint64_t>(kp.P) < 3u * grid_lanes);
  // The previous frame of this context still running (its end event pending): frames are
  // being streamed, and this trace shares the CUs with the previous frame's trace or sum
  const bool prev_in_flight = !dry && c->pending && hipEventQuery(c->ev1) == hipErrorNotReady;
  // one frame of memory: the first frame of a burst that follows a host wait (a timed region
  // after its warm-up) still overlaps; a caller that waits for every frame (update()) never does
  const bool stream_mode = prev_in_flight || c->streaming;
  if (!dry) c->streaming = prev_in_flight;
  const size_t slot_bytes = per_block * nb_pass;
  // a new layout (slot count or size, or not pipelined): every earlier frame must have been
  // summed before this one reuses the buffers; in one layout only this slot's last user
  const bool relayout = !fpipe || nfs != c->fs_n || slot_bytes != c->fs_bytes;
  if (relayout) c->frame_slot = 0;
  const int fs = fpipe ? c->frame_slot % nfs : 0;
  unsigned long long* cnt = c->d_cnt + kCntWords * fs;
  const int slots = passes > 1 ? 2 : fpipe ? nfs : 1;
  if (kp.P && nb_pass && slot_bytes * slots > c->cap_samples) {
    if (c->d_samples) HIPCHK(hipFree(c->d_samples));
    c->d_samples = nullptr;
    c->cap_samples = 0;
    HIPCHK(hipMalloc(&c->d_samples, slot_bytes * slots));
    c->cap_samples = slot_bytes * slots;
  }
  const size_t running_bytes = static_cast<size_t>(kp.P) * 3 * sizeof(float);
  if (passes > 1 && running_bytes > c->cap_running) {
    if (c->d_running) HIPCHK(hipFree(c->d_running));
    c->d_running = nullptr;
    c->cap_running = 0;
    HIPCHK(hipMalloc(&c->d_running, running_bytes));
    c->cap_running = running_bytes;
  }
  while (c->ev_sum.size() < static_cast<size_t>(passes > 0 ? passes : 1)) {
    hipEvent_t e;
    HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->ev_sum.push_back(e);
  }
  while (c->ev_trace.size() < 2u * static_cast<size_t>(passes > 0 ? passes : 1)) {
    hipEvent_t e;
    HIPCHK(hipEventCreate(&e));
    c->ev_trace.push_back(e);
  }
  const size_t n_att = dc->n <= kAttLds ? dc->n : 0u;
  const size_t stack_bytes = nibble ? 0u
                           : defer ? kSmallDepth * kBlock * sizeof(uint8_t)
                           : small_depth ? kSmallDepth * kBlock * sizeof(uint16_t)
                                         : static_cast<size_t>(p->max_depth ? p->max_depth : 1u) * kBlock *
                                               sizeof(uint32_t);
  const size_t n_rec = dc->n <= kRecLds ? dc->n : 0u;
  const size_t stage_n = stage_samples(use_bvh, nibble);
  const size_t lds = (stage_n > 1 && (!use_bvh || nibble) ? kBlock * stage_n * wps * sizeof(float) : 0u) +
                     (n_att ? n_att + 1 : 0) * 16 +
                     n_rec * 64 + stack_bytes +
                     (use_bvh ? (dc->bvh_levels + 1u) * kBlock * sizeof(uint32_t) : 0u);  // + the sentinel row
  // the scene-specialised kernel (jit.h): list-loop scenes of <= kJitMaxPrims primitives,
  // when the caller asks (FR_FLAG_SCENE_JIT; FR_SCENE_JIT=1 / 0 forces it on / off)
  JitReq jr;
  jr.device = c->device;
  jr.dc = dc;
  {
    const char* je = getenv("FR_SCENE_JIT");
    const bool want = je && *je ? strcmp(je, "0") != 0 : (p->flags & FR_FLAG_SCENE_JIT) != 0;
#if defined(FR_DIAG)
    const bool build_ok = false;  // diagnostics builds keep their device globals in this library
#else
    const bool build_ok = true;
#endif
    jr.on = want && build_ok && !use_bvh && dc->n >= 1 && dc->n <= kJitMaxPrims;
    // prepare, FR_FLAG_SCENE_JIT_WAIT and the environment's FR_SCENE_JIT=1 wait for the
    // compile; plain FR_FLAG_SCENE_JIT renders run the compiled-in kernel until it is done
    jr.wait = dry || (p->flags & FR_FLAG_SCENE_JIT_WAIT) != 0 || (je && *je && strcmp(je, "0") != 0);
    jr.cached_only = !jr.wait && (p->flags & FR_FLAG_SCENE_JIT_CACHED) != 0;
  }
  KWork kw;
  kw.counters = cnt;
  // the scene-specialised kernel is looked up here (loaded, or compiled when waiting),
  // before anything is enqueued, so a first frame's events do not span the compile
  JitStats jit_got{};
  const uint32_t jc_flags = kp.flags & (KF_DEFER | KF_NIBBLE | KF_DIFFUSE | FR_FLAG_MT_BANDS);
  if (jr.on && kp.P && c->jc_fn && c->jc_uid == dc->uid && c->jc_flags == jc_flags && c->jc_small == small_depth) {
    jr.resolved = true;
    jr.fn = c->jc_fn;
    jr.pin = c->jc_pin;
    jit_got.reused = 1;
    jit_got.state = FR_JIT_USED;
  } else if (jr.on && kp.P) {
    JitReq pre = jr;
    pre.dry = true;
    uint32_t blocks = 0;
    int occ = 0;
    const Grid grid{1, c->num_cus, &occ, &blocks, 0};
    rc = launch_trace(dc->kinds, dc->has_plane, use_bvh, small_depth, grid, lds, c->stream, KArgs{ks, kc, kp, kw},
                      &pre);
    if (rc) return rc;
    jit_got = pre.stats;
    jr.resolved = pre.resolved;
    jr.fn = pre.fn;
    jr.pin = pre.stats.pin;
    c->jc_fn = pre.fn;  // null (pending or failed): looked up again next render
    c->jc_pin = pre.stats.pin;
    c->jit_stats.pin.reset();
    c->jc_uid = dc->uid;
    c->jc_flags = jc_flags;
    c->jc_small = small_depth;
  }
  const int jit_state = jr.on && kp.P ? jit_got.state : FR_JIT_OFF;
  if (dry) {
    c->jit_used = jr.on && kp.P && jr.fn != nullptr;
    c->jit_stats = jit_got;
    c->jit_state = jit_state;
    return FR_OK;
  }
  c->t0 = std::chrono::steady_clock::now();
  // the last frame that used this slot's counters and samples (or, after a layout change,
  // every earlier frame) has been summed
#ifndef FR_SETUP_ON_TRACE_STREAM
#define FR_SETUP_ON_TRACE_STREAM 1
#endif
  // The frame's setup (slot wait, counter clear, start events) goes on the stream its trace
  // runs on: with overlapping traces (stream2 every other frame) a setup on c->stream would
  // wait behind the previous frame's whole trace there, and so would this frame's trace.
  hipStream_t setup = c->stream;
  if (FR_SETUP_ON_TRACE_STREAM && fpipe && fpipe_overlap && c->frame_parity) setup = c->stream2;
  for (int k = 0; k < fr_ctx::kFrameSlots; ++k)
    if (c->fslot_used[k] && (k == fs || relayout)) HIPCHK(hipStreamWaitEvent(setup, c->ev_fslot[k], 0));
  c->fs_n = nfs;
  c->fs_bytes = slot_bytes;
  HIPCHK(hipMemsetAsync(cnt, 0, kCntWords * sizeof(unsigned long long), setup));
#ifdef FR_DIAG
  {
    const unsigned long long z[2] = {0, 0};
    HIPCHK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_fr_diag_lens), z, sizeof(z), 0, hipMemcpyHostToDevice, setup));
    HIPCHK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_fr_diag_rus), z, sizeof(z), 0, hipMemcpyHostToDevice, setup));
    void* tc = nullptr;
    HIPCHK(hipGetSymbolAddress(&tc, HIP_SYMBOL(g_fr_tb_cost)));
    HIPCHK(hipMemsetAsync(tc, 0, (1u << 20) * sizeof(unsigned int), setup));
  }
#endif
  HIPCHK(hipEventRecord(c->ev0, setup));
  if (c->log_on) HIPCHK(log_start(c, 1, setup));
  HIPCHK(hipEventRecord(c->ev_start, setup));
  if (setup != c->stream2) HIPCHK(hipStreamWaitEvent(c->stream2, c->ev_start, 0));
  HIPCHK(hipStreamWaitEvent(c->stream_sum, c->ev_start, 0));
  const uint32_t sum_blocks = (kp.P + kSumThreads - 1u) / kSumThreads;
  int traced = 0;  // trace launches whose events were recorded
  int summed = 0;
  for (int pass = 0; pass < passes || (pass == 0 && kp.P); ++pass) {
    const int slot = fpipe ? fs : pass % 2;
    // one trace stream for pipelined frames: frame k+1's trace follows frame k's trace
    hipStream_t ts = fpipe ? (fpipe_overlap && c->frame_parity ? c->stream2 : c->stream) : slot ? c->stream2 : c->stream;
    float* samples = c->d_samples ? c->d_samples + static_cast<size_t>(slot) * (slot_bytes / sizeof(float)) : nullptr;
    kp.b0 = static_cast<uint32_t>(pass) * nb_pass;
    kp.nb = pass < passes ? min(nb_pass, nblocks - kp.b0) : 0u;
    kp.n_items = kp.nb * kp.P;
    kp.n_coarse = kp.n_items;
    kp.b_fine = 0;
    if (kFineSub > 1 && nblocks > 1 && kp.nb && kp.b0 + kp.nb == nblocks) {
      // the pixels' last block, as sub-blocks of kFineSamples: the queue's last items
      const uint32_t n_last = p->spp - (nblocks - 1u) * kBlockSamples;
      kp.n_coarse = (kp.nb - 1u) * kp.P;
      kp.b_fine = nblocks - 1u;
      kp.n_items = kp.n_coarse + ((n_last + kFineSamples - 1u) / kFineSamples) * kp.P;
    }
    if (kp.n_items) {
      if (pass >= 2) HIPCHK(hipStreamWaitEvent(ts, c->ev_sum[pass - 2], 0));  // the slot's last reader is done
      kw.queue = reinterpret_cast<uint32_t*>(cnt + 31 - (fpipe ? 0 : slot));
      kw.samples = samples;
      // persistent grid: the resident workgroup count (launch_persistent)
      uint32_t blocks = 0;
      Grid grid{(static_cast<uint64_t>(kp.n_items) + kBlock - 1u) / kBlock, c->num_cus, &c->occupancy, &blocks,
                use_bvh && !nibble && stage_n > 1 && !FR_BVH_RSTAGE ? kBlock * stage_n * 3 * sizeof(float) : 0u};
      // pipelined frames leave room on every CU for the previous frame's sum workgroups:
      // one slot at N = 1 (two cost 6 %); until round 5 two for shards
      // whose traces overlap (shard 1/8 2.23 -> 2.18 ms per frame against one).
      // Round 6: overlapping traces of streamed frames take half the CU slots each (reserve
      // 4 of 8), so two frames' traces run side by side and each fills the other's drain:
      // shards of 8 stream at 1.81 ms per frame against 1.90 with reserve 2, of 4 at 3.60
      // against 3.70, of 2 at 7.21 against 7.30 (profiles/r06i_*, r06j_*). A frame whose
      // predecessor has finished shares the CUs with nothing: no reserve.
      if (fpipe) {
        const char* r = getenv("FR_FRAME_PIPE_RESERVE");
        grid.reserve = r ? static_cast<uint32_t>(atoi(r)) : !stream_mode ? 0u : fpipe_overlap ? 4u : 1u;
      }
      unsigned long long* wcnt = c->d_wcnt + static_cast<size_t>(slot) * 3 * kMaxWgPerCu * (kBlock / 64u) * c->num_cus;
      kw.wave_counters = wcnt;
#ifndef FR_QUEUE_MEMSET
#define FR_QUEUE_MEMSET 0
#endif
      // a pipelined frame's queue head is cnt[31], cleared with its counters above (before
      // ev_start, which stream2 waits for); passes of a multi-pass frame reuse two heads
      if (!fpipe || FR_QUEUE_MEMSET) HIPCHK(hipMemsetAsync(kw.queue, 0, sizeof(uint32_t), ts));
      HIPCHK(hipEventRecord(c->ev_trace[2 * traced], ts));
      if (c->log_on) HIPCHK(log_start(c, 0, ts));
      rc = launch_trace(dc->kinds, dc->has_plane, use_bvh, small_depth, grid, lds, ts, KArgs{ks, kc, kp, kw}, &jr);
      if (rc) return rc;
      HIPCHK(hipGetLastError());
      HIPCHK(hipEventRecord(c->ev_trace[2 * traced + 1], ts));
      if (c->log_on) HIPCHK(log_end(c, 0, ts));
      HIPCHK(hipStreamWaitEvent(c->stream_sum, c->ev_trace[2 * traced + 1], 0));
      // on the sum stream, after the trace: the frame's end (ev1 on c->stream) waits for
      // the sums, so fr_ctx_sync reads d_cnt after every pass's reduce, and the next
      // frame's d_cnt memset (c->stream) cannot overtake a reduce of this one
      hipLaunchKernelGGL(reduce_counters, dim3(1), dim3(256), 0, c->stream_sum, wcnt, blocks * (kBlock / 64u),
                         cnt);
      HIPCHK(hipGetLastError());
      ++traced;
    }
    const int first = pass == 0, last = pass + 1 >= passes;
    if (first && c->copy_pending) HIPCHK(hipStreamWaitEvent(c->stream_sum, c->ev_copy, 0));  // last gather done
    const int sum_kind = wps == 3 && kSkyDefer && nibble ? 1 : 0;
    // (BVH kernels with 8-B records store attenuation classes: the class table)
    HIPCHK(launch_sum(wps, sum_kind, sum_blocks ? sum_blocks : 1u, c->stream_sum, kp, samples, c->d_running,
                      c->d_mean, c->d_u8, first, last,
                      bvh_nib ? reinterpret_cast<const float4*>(b + dc->off_acls_att) : ks.att,
                      bvh_nib ? dc->n_aclass : dc->n));
    HIPCHK(hipEventRecord(c->ev_sum[pass], c->stream_sum));
    summed = pass + 1;
    if (last) break;
  }
  // frame end: on the context's stream (the next frame's trace waits for this one's sums),
  // or, pipelined, on the sum stream (the next frame's trace starts when this trace ends)
  hipStream_t end_stream = c->stream;
  if (fpipe)
    end_stream = c->stream_sum;
  else if (summed)
    HIPCHK(hipStreamWaitEvent(c->stream, c->ev_sum[summed - 1], 0));
  HIPCHK(hipEventRecord(c->ev_fslot[fs], end_stream));
  c->fslot_used[fs] = true;
  c->last_cnt = cnt;
  if (fpipe) {
    c->frame_slot = (fs + 1) % nfs;
    c->frame_parity ^= 1;
  }
  c->passes = traced;
  c->jit_used = jr.used;
  c->jit_stats = jit_got;
  c->jit_state = jit_state;
  HIPCHK(hipEventRecord(c->ev1, end_stream));
  if (c->log_on) HIPCHK(log_end(c, 1, end_stream));
  c->last = *p;
  c->last_n = dc->n;
  c->pending = true;
  return FR_OK;
}

int fr_ctx_sync(fr_ctx* c, fr_stats* st) {
  if (!c) return set_error(FR_EARG, "fr_ctx_sync: null ctx");
  SET_DEVICE(c->device);
  HIPCHK(hipStreamSynchronize(c->stream));
  if (!c->pending) return set_error(FR_EARG, "fr_ctx_sync: nothing rendered");
  HIPCHK(hipEventSynchronize(c->ev1));  // the frame's end (on the sum stream when pipelined)
  if (st) {
    unsigned long long cnt[kCntWords] = {};
    HIPCHK(hipMemcpy(cnt, c->last_cnt, sizeof(cnt), hipMemcpyDeviceToHost));
#ifdef FR_PROF
    {
      double tot = 0;
      for (int k = 0; k < PF_N; ++k) tot += static_cast<double>(cnt[20 + k]);
      fprintf(stderr, "FR_PROF {\"claim\": %.4f, \"reject\": %.4f, \"hit\": %.4f, \"shade\": %.4f, \"end\": %.4f, "
              "\"wave_cycles\": %.4e}\n", cnt[20] / tot, cnt[21] / tot, cnt[22] / tot, cnt[23] / tot, cnt[24] / tot, tot);
    }
#endif
#ifdef FR_SECCNT
    fprintf(stderr, "FR_SECCNT [");
    for (int k = 0; k < SC_N; ++k) fprintf(stderr, k ? ", %llu" : "%llu", cnt[4 + k]);
    fprintf(stderr, "]\nFR_SECLANES [");
    for (int k = 0; k < SC_N; ++k) fprintf(stderr, k ? ", %llu" : "%llu", cnt[32 + k]);
    fprintf(stderr, "]\n");
#endif
#ifdef FR_DIAG
    unsigned long long dl[2], dr[2];
    HIPCHK(hipMemcpyFromSymbol(dl, HIP_SYMBOL(g_fr_diag_lens), sizeof(dl)));
    HIPCHK(hipMemcpyFromSymbol(dr, HIP_SYMBOL(g_fr_diag_rus), sizeof(dr)));
    fprintf(stderr,
            "FR_DIAG {\"iter_w\": %llu, \"regen_w\": %llu, \"regen_l\": %llu, \"hit_w\": %llu, \"end_w\": %llu, "
            "\"end_l\": %llu, \"unwind_w\": %llu, \"unwind_l\": %llu, \"lens_w\": %llu, \"lens_l\": %llu, "
            "\"rus_w\": %llu, \"rus_l\": %llu, \"merged_w\": %llu, \"merged_l\": %llu, \"segments\": %llu, "
            "\"hits\": %llu, \"node_w\": %llu, \"node_l\": %llu, \"leaf_w\": %llu, \"leaf_l\": %llu, "
            "\"node_coh_w\": %llu, \"node_u2_w\": %llu, \"node_u34_w\": %llu, \"node_primary_l\": %llu}\n",
            cnt[4 + DG_ITER], cnt[4 + DG_REGEN_W], cnt[4 + DG_REGEN_L], cnt[4 + DG_HIT_W], cnt[4 + DG_END_W],
            cnt[4 + DG_END_L], cnt[4 + DG_UNW_W], cnt[4 + DG_UNW_L], dl[0], dl[1], dr[0], dr[1], cnt[4 + DG_LENS_W],
            cnt[4 + DG_LENS_L], cnt[0], cnt[1], cnt[4 + DG_NODE_W], cnt[4 + DG_NODE_L], cnt[4 + DG_LEAF_W],
            cnt[4 + DG_LEAF_L], cnt[4 + DG_NCOH_W], cnt[4 + DG_NU2_W], cnt[4 + DG_NU4_W], cnt[4 + DG_NPRIM_L]);
    if (const char* path = getenv("FR_DIAG_COST")) {
      std::vector<unsigned int> tc(1u << 20);
      HIPCHK(hipMemcpyFromSymbol(tc.data(), HIP_SYMBOL(g_fr_tb_cost), tc.size() * 4));
      if (FILE* f = fopen(path, "wb")) {
        fwrite(tc.data(), 4, tc.size(), f);
        fclose(f);
      }
    }
    if (const char* path = getenv("FR_DIAG_TIMES")) {
      std::vector<unsigned long long> wt(2 * 65536);
      HIPCHK(hipMemcpyFromSymbol(wt.data(), HIP_SYMBOL(g_fr_wave_times), wt.size() * 8));
      std::vector<unsigned long long> wd(65536);
      HIPCHK(hipMemcpyFromSymbol(wd.data(), HIP_SYMBOL(g_fr_wave_drain), wd.size() * 8));
      wt.insert(wt.end(), wd.begin(), wd.end());
      if (const char* pi = getenv("FR_DIAG_ITERS")) {
        std::vector<unsigned long long> ti(1024 * 1024);
        HIPCHK(hipMemcpyFromSymbol(ti.data(), HIP_SYMBOL(g_fr_iter_times), ti.size() * 8));
        if (FILE* f = fopen(pi, "wb")) {
          fwrite(ti.data(), 8, ti.size(), f);
          fclose(f);
        }
      }
      std::vector<unsigned int> wi(2 * 65536);
      HIPCHK(hipMemcpyFromSymbol(wi.data(), HIP_SYMBOL(g_fr_wave_iters), wi.size() * 4));
      for (size_t k = 0; k < wi.size(); k += 2) wt.push_back((static_cast<unsigned long long>(wi[k + 1]) << 32) | wi[k]);
      if (FILE* f = fopen(path, "wb")) {
        fwrite(wt.data(), 8, wt.size(), f);
        fclose(f);
      }
    }
#endif
    float ms = 0.0f;
    HIPCHK(hipEventElapsedTime(&ms, c->ev0, c->ev1));
    const fr_params& p = c->last;
    const uint32_t strips = (p.height + kStripRows - 1) / kStripRows;
    uint64_t rows = 0, traced_rows = 0;
    // render_mt never traces the rows past 4 * (H / 4) (tracer.rs:87)
    const uint32_t mt_end = (p.flags & FR_FLAG_MT_BANDS) ? (p.height / 4u) * 4u : p.height;
    for (uint32_t k = p.shard_index; k < strips; k += p.shard_count) {
      const uint32_t r0 = k * kStripRows, r1 = r0 + kStripRows < p.height ? r0 + kStripRows : p.height;
      rows += r1 - r0;
      traced_rows += r1 <= mt_end ? r1 - r0 : r0 < mt_end ? mt_end - r0 : 0u;
    }
    st->segments = cnt[0];
    st->hits = cnt[1];
    st->samples = rows * p.width * static_cast<uint64_t>(p.spp);
    st->prim_tests = cnt[0] * static_cast<uint64_t>(c->last_n);
    st->kernel_ms = ms;
    double tms = 0.0;
    for (int i = 0; i < c->passes; ++i) {
      float t = 0.0f;
      HIPCHK(hipEventElapsedTime(&t, c->ev_trace[2 * i], c->ev_trace[2 * i + 1]));
      tms += t;
    }
    st->trace_ms = tms;
    st->trace_launches = static_cast<uint32_t>(c->passes);
    st->occupancy = static_cast<uint32_t>(c->occupancy);
    // every path traces one segment more than it scatters (tracer.rs:189-210: each scatter
    // is followed by one more get_color), so the kernel counts segments and hits only
    st->scatters = cnt[0] - traced_rows * p.width * static_cast<uint64_t>(p.spp);
    st->total_ms =
        std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - c->t0).count();
  }
  return FR_OK;
}

// Enqueues the D2H copies of this shard's rows of the last render on `st`.
static int enqueue_download(fr_ctx* c, hipStream_t st, float* mean_rgb, uint8_t* rgb8) {
  const fr_params& p = c->last;
  const uint32_t strips = (p.height + kStripRows - 1) / kStripRows;
  const size_t row_f = static_cast<size_t>(p.width) * 3;  // elements per row
  if (p.shard_count == 1) {  // the whole image: one contiguous copy per output
    const size_t n = static_cast<size_t>(p.height) * row_f;
    if (mean_rgb) HIPCHK(hipMemcpyAsync(mean_rgb, c->d_mean, n * 4, hipMemcpyDeviceToHost, st));
    if (rgb8) HIPCHK(hipMemcpyAsync(rgb8, c->d_u8, n, hipMemcpyDeviceToHost, st));
    return FR_OK;
  }
  // full strips of this shard form a strided 2-D region; the trailing partial strip is separate
  uint32_t full = 0, partial = 0;
  for (uint32_t k = p.shard_index; k < strips; k += p.shard_count) {
    if ((k + 1) * kStripRows <= p.height)
      ++full;
    else
      partial = k;
  }
  const size_t first = static_cast<size_t>(p.shard_index) * kStripRows * row_f;
  const size_t pitch = static_cast<size_t>(p.shard_count) * kStripRows * row_f;
  const size_t width = kStripRows * row_f;
  const bool has_partial = (p.height % kStripRows) != 0 && (strips - 1) % p.shard_count == p.shard_index;
  if (mean_rgb) {
    if (full)
      HIPCHK(hipMemcpy2DAsync(mean_rgb + first, pitch * 4, c->d_mean + first, pitch * 4, width * 4, full,
                              hipMemcpyDeviceToHost, st));
    if (has_partial) {
      const size_t o = static_cast<size_t>(partial) * kStripRows * row_f;
      HIPCHK(hipMemcpyAsync(mean_rgb + o, c->d_mean + o, (p.height - partial * kStripRows) * row_f * 4,
                            hipMemcpyDeviceToHost, st));
    }
  }
  if (rgb8) {
    if (full)
      HIPCHK(hipMemcpy2DAsync(rgb8 + first, pitch, c->d_u8 + first, pitch, width, full, hipMemcpyDeviceToHost, st));
    if (has_partial) {
      const size_t o = static_cast<size_t>(partial) * kStripRows * row_f;
      HIPCHK(hipMemcpyAsync(rgb8 + o, c->d_u8 + o, (p.height - partial * kStripRows) * row_f,
                            hipMemcpyDeviceToHost, st));
    }
  }
  return FR_OK;
}

int fr_ctx_download(fr_ctx* c, float* mean_rgb, uint8_t* rgb8) {
  if (!c || !c->pending) return set_error(FR_EARG, "fr_ctx_download: nothing rendered");
  SET_DEVICE(c->device);
  HIPCHK(hipStreamWaitEvent(c->stream, c->ev1, 0));  // the last render's end (its sums)
  const int rc = enqueue_download(c, c->stream, mean_rgb, rgb8);
  if (rc) return rc;
  HIPCHK(hipStreamSynchronize(c->stream));
  return FR_OK;
}

int fr_ctx_download_async(fr_ctx* c, float* mean_rgb, uint8_t* rgb8) {
  if (!c || !c->pending) return set_error(FR_EARG, "fr_ctx_download_async: nothing rendered");
  SET_DEVICE(c->device);
  HIPCHK(hipStreamWaitEvent(c->stream_copy, c->ev1, 0));  // after the last render's sum
  const int rc = enqueue_download(c, c->stream_copy, mean_rgb, rgb8);
  if (rc) return rc;
  HIPCHK(hipEventRecord(c->ev_copy, c->stream_copy));
  c->copy_pending = true;
  return FR_OK;
}

int fr_ctx_wait(fr_ctx* c) {
  if (!c) return set_error(FR_EARG, "fr_ctx_wait: null ctx");
  SET_DEVICE(c->device);
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipStreamSynchronize(c->stream2));
  HIPCHK(hipStreamSynchronize(c->stream_sum));
  HIPCHK(hipStreamSynchronize(c->stream_copy));
  return FR_OK;
}

int fr_host_alloc(size_t bytes, void** out) {
  if (!out) return set_error(FR_EARG, "fr_host_alloc: null output");
  *out = nullptr;
  if (hipHostMalloc(out, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess || !*out)
    return set_error(FR_ENOMEM, "hipHostMalloc(%zu) failed", bytes);
  return FR_OK;
}

void fr_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

int fr_ctx_device_buffers(fr_ctx* c, float** d_mean, uint8_t** d_u8) {
  if (!c) return set_error(FR_EARG, "fr_ctx_device_buffers: null ctx");
  if (d_mean) *d_mean = c->d_mean;
  if (d_u8) *d_u8 = c->d_u8;
  return FR_OK;
}

int fr_render_hip(fr_scene* scene, const fr_camera* cam, const fr_params* params, int device, float* mean_rgb,
                  uint8_t* rgb8, fr_stats* stats) {
  fr_ctx* c = nullptr;
  int rc = fr_ctx_create(device, nullptr, &c);
  if (rc) return rc;
  fr_params p = *params;
  if (rgb8) p.flags |= FR_FLAG_WRITE_U8;
  rc = fr_ctx_render(c, scene, cam, &p);
  if (!rc) rc = fr_ctx_sync(c, stats);
  if (!rc) rc = fr_ctx_download(c, mean_rgb, rgb8);
  fr_ctx_free(c);
  return rc;
}

// Test hook, no device needed: the run-time build of the headline specialisation (all
// boxes, <= 15 primitives, diffuse, depth <= 8) for `n` 64-B records compiles for `arch`.
// targs: the 8 template arguments of another specialisation (NULL: the headline's).
int fr_selftest_jit(const char* arch, const uint32_t* rec, uint32_t n, const int* targs_in, size_t* code_bytes,
                    double* ms) {
  if (!arch || !rec || n == 0 || n > kJitMaxPrims) return set_error(FR_EARG, "fr_selftest_jit: bad arguments");
  int targs[8] = {KS_AABB, 0, FR_KREJ_NIB, static_cast<int>(kSmallDepth), 0, 0, 2, 1};
  if (targs_in) memcpy(targs, targs_in, sizeof targs);
  char name[160];
  snprintf(name, sizeof name, "fr::trace_kernel<%d, %s, %d, %d, %s, %s, %d, %d>", targs[0],
           targs[1] ? "true" : "false", targs[2], targs[3], targs[4] ? "true" : "false", targs[5] ? "true" : "false",
           targs[6], targs[7]);
  const bool tbool[8] = {false, true, false, false, true, true, false, false};
  const JitSpec spec{name, targs, tbool, 8, jit_defines(), rec, n};
  return jit_compile_probe(arch, spec, code_bytes, ms);
}

int fr_ctx_jit_info(fr_ctx* c, int* used, double* ms, int* compiled) {
  if (!c) return set_error(FR_EARG, "fr_ctx_jit_info: null ctx");
  if (used) *used = c->jit_used ? 1 : 0;
  if (ms) *ms = c->jit_state != FR_JIT_OFF ? c->jit_stats.ms : 0.0;
  if (compiled) *compiled = c->jit_state != FR_JIT_OFF ? c->jit_stats.compiled : 0;
  return FR_OK;
}

int fr_ctx_jit_state(fr_ctx* c, int* state) {
  if (!c || !state) return set_error(FR_EARG, "fr_ctx_jit_state: null argument");
  *state = c->jit_state;
  if (c->jit_state == FR_JIT_FAILED) set_error(FR_EHIP, "%s", c->jit_stats.error.c_str());
  return FR_OK;
}

int fr_jit_wait(void) { return jit_wait_all(); }

int fr_ctx_trace_log(fr_ctx* c, int enable) {
  if (!c) return set_error(FR_EARG, "fr_ctx_trace_log: null ctx");
  if (enable) {
    SET_DEVICE(c->device);
    // the pairs of an earlier log may still be pending on the streams (a pipelined render
    // records its end on the sum stream): drain them before their events are recorded again
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipStreamSynchronize(c->stream2));
    HIPCHK(hipStreamSynchronize(c->stream_sum));
    c->log_n[0] = c->log_n[1] = 0;
  }
  c->log_on = enable != 0;
  return FR_OK;
}

int fr_ctx_trace_log_read(fr_ctx* c, int which, double* ms, uint32_t cap, uint32_t* n) {
  if (!c || !n || which < 0 || which > 3) return set_error(FR_EARG, "fr_ctx_trace_log_read: bad argument");
  SET_DEVICE(c->device);
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipStreamSynchronize(c->stream2));
  HIPCHK(hipStreamSynchronize(c->stream_sum));  // a pipelined render's end event is recorded there
  // which 0 / 1: durations of the trace launches / renders; 2 / 3: their start and end times
  // (two values each) from the first logged trace launch's start (a timeline)
  const int w = which & 1;
  *n = static_cast<uint32_t>(c->log_n[w]);
  for (size_t i = 0; i < c->log_n[w] && ms; ++i) {
    if (which < 2) {
      if (i >= cap) break;
      float t = 0.0f;
      HIPCHK(hipEventElapsedTime(&t, c->log_ev[w][2 * i], c->log_ev[w][2 * i + 1]));
      ms[i] = t;
    } else {
      if (2 * i + 1 >= cap || c->log_n[0] == 0) break;
      float a = 0.0f, b = 0.0f;
      HIPCHK(hipEventElapsedTime(&a, c->log_ev[0][0], c->log_ev[w][2 * i]));
      HIPCHK(hipEventElapsedTime(&b, c->log_ev[0][0], c->log_ev[w][2 * i + 1]));
      ms[2 * i] = a;
      ms[2 * i + 1] = b;
    }
  }
  return FR_OK;
}

}  // extern "C"

// ---- multi-device context (render_mt's row tiling over devices, tracer.rs:83-134) ----
// One fr_ctx per entry of the device list (duplicates allowed: two contexts on one device
// rehearse a two-device run), each rendering shard i of n of every frame; the shards'
// strips land in one page-locked host frame by asynchronous D2H copies, one per context.
// Everything is allocated at creation or on a frame of a larger size; a frame of the same
// size allocates nothing.
struct fr_mctx {
  std::vector<fr_ctx*> ctx;
  float* h_mean = nullptr;  // pinned full frame: W x H x 3 f32, then W x H x 3 u8
  uint8_t* h_u8 = nullptr;
  size_t cap_pixels = 0;
  uint32_t width = 0, height = 0;
  bool pending = false;
  std::chrono::steady_clock::time_point t0;
};

extern "C" {

void fr_mctx_free(fr_mctx* m) {
  if (!m) return;
  for (fr_ctx* c : m->ctx) fr_ctx_free(c);  // each drains its streams first
  if (m->h_mean) (void)hipHostFree(m->h_mean);
  delete m;
}

int fr_mctx_create(const int* devices, int n, fr_mctx** out) {
  if (!devices || n < 1 || !out) return set_error(FR_EARG, "fr_mctx_create: bad arguments");
  *out = nullptr;
  fr_mctx* m = new fr_mctx();
  for (int i = 0; i < n; ++i) {
    fr_ctx* c = nullptr;
    const int rc = fr_ctx_create(devices[i], nullptr, &c);
    if (rc) {
      const std::string msg = fr_last_error();
      fr_mctx_free(m);
      return set_error(rc, "fr_mctx_create: entry %d (device %d): %s", i, devices[i], msg.c_str());
    }
    m->ctx.push_back(c);
  }
  *out = m;
  return FR_OK;
}

int fr_mctx_count(const fr_mctx* m) { return m ? static_cast<int>(m->ctx.size()) : 0; }

int fr_mctx_ctx(fr_mctx* m, int i, fr_ctx** out) {
  if (!m || !out || i < 0 || i >= static_cast<int>(m->ctx.size())) return set_error(FR_EARG, "fr_mctx_ctx: bad index");
  *out = m->ctx[i];
  return FR_OK;
}

int fr_mctx_render(fr_mctx* m, fr_scene* scene, const fr_camera* cam, const fr_params* params) {
  if (!m || !scene || !cam || !params) return set_error(FR_EARG, "fr_mctx_render: null argument");
  const int n = static_cast<int>(m->ctx.size());
  fr_params p = *params;
  p.shard_count = static_cast<uint32_t>(n);
  p.shard_index = 0;
  int rc = check_params(&p);
  if (rc) return rc;
  const size_t pixels = static_cast<size_t>(p.width) * p.height;
  if (pixels > m->cap_pixels) {
    // a larger frame: the previous frame's gathers may still write the old host frame
    for (fr_ctx* c : m->ctx)
      if ((rc = fr_ctx_wait(c))) return rc;
    if (m->h_mean) HIPCHK(hipHostFree(m->h_mean));
    m->h_mean = nullptr;
    m->h_u8 = nullptr;
    m->cap_pixels = 0;
    void* h = nullptr;
    HIPCHK(hipHostMalloc(&h, pixels * 3 * (sizeof(float) + 1), hipHostMallocDefault));
    m->h_mean = static_cast<float*>(h);
    m->h_u8 = reinterpret_cast<uint8_t*>(m->h_mean + pixels * 3);
    m->cap_pixels = pixels;
  }
  m->width = p.width;
  m->height = p.height;
  m->t0 = std::chrono::steady_clock::now();
  // enqueue every shard and its gather, then return: the devices run concurrently
  for (int i = 0; i < n; ++i) {
    p.shard_index = static_cast<uint32_t>(i);
    if ((rc = fr_ctx_render(m->ctx[i], scene, cam, &p))) return set_error(rc, "shard %d: %s", i, fr_last_error());
    if ((rc = fr_ctx_download_async(m->ctx[i], m->h_mean, (p.flags & FR_FLAG_WRITE_U8) ? m->h_u8 : nullptr)))
      return set_error(rc, "shard %d: %s", i, fr_last_error());
  }
  m->pending = true;
  return FR_OK;
}

int fr_mctx_sync(fr_mctx* m, fr_stats* stats) {
  if (!m) return set_error(FR_EARG, "fr_mctx_sync: null mctx");
  if (!m->pending) return set_error(FR_EARG, "fr_mctx_sync: nothing rendered");
  fr_stats agg;
  memset(&agg, 0, sizeof(agg));
  for (size_t i = 0; i < m->ctx.size(); ++i) {
    fr_stats st;
    int rc = fr_ctx_sync(m->ctx[i], &st);
    if (!rc) rc = fr_ctx_wait(m->ctx[i]);  // the shard's gather has landed
    if (rc) return set_error(rc, "shard %zu: %s", i, fr_last_error());
    agg.segments += st.segments;
    agg.hits += st.hits;
    agg.samples += st.samples;
    agg.prim_tests += st.prim_tests;
    agg.scatters += st.scatters;
    agg.kernel_ms = std::max(agg.kernel_ms, st.kernel_ms);  // the slowest shard
    agg.trace_ms = std::max(agg.trace_ms, st.trace_ms);
    agg.trace_launches = std::max(agg.trace_launches, st.trace_launches);
    agg.occupancy = st.occupancy;
  }
  agg.total_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - m->t0).count();
  if (stats) *stats = agg;
  return FR_OK;
}

int fr_mctx_frame(fr_mctx* m, const float** mean_rgb, const uint8_t** rgb8) {
  if (!m || !m->pending) return set_error(FR_EARG, "fr_mctx_frame: nothing rendered");
  if (mean_rgb) *mean_rgb = m->h_mean;
  if (rgb8) *rgb8 = m->h_u8;
  return FR_OK;
}

int fr_mctx_download(fr_mctx* m, float* mean_rgb, uint8_t* rgb8) {
  if (!m || !m->pending) return set_error(FR_EARG, "fr_mctx_download: nothing rendered");
  for (fr_ctx* c : m->ctx) {
    const int rc = fr_ctx_wait(c);
    if (rc) return rc;
  }
  const size_t n = static_cast<size_t>(m->width) * m->height * 3;
  if (mean_rgb) memcpy(mean_rgb, m->h_mean, n * sizeof(float));
  if (rgb8) memcpy(rgb8, m->h_u8, n);
  return FR_OK;
}

int fr_render_hip_multi(fr_scene* scene, const fr_camera* cam, const fr_params* params, int n_gpus,
                        float* mean_rgb, uint8_t* rgb8, fr_stats* stats) {
  if (!params || n_gpus < 1) return set_error(FR_EARG, "fr_render_hip_multi: bad arguments");
  int avail = 0;
  if (hipGetDeviceCount(&avail) != hipSuccess || avail < n_gpus)
    return set_error(FR_ENODEV, "fr_render_hip_multi: %d devices requested, %d present", n_gpus, avail);
  std::vector<int> devs(n_gpus);
  for (int g = 0; g < n_gpus; ++g) devs[g] = g;
  fr_mctx* m = nullptr;
  int rc = fr_mctx_create(devs.data(), n_gpus, &m);
  if (rc) return rc;
  fr_params p = *params;
  if (rgb8) p.flags |= FR_FLAG_WRITE_U8;
  rc = fr_mctx_render(m, scene, cam, &p);
  if (!rc) rc = fr_mctx_sync(m, stats);
  if (!rc) rc = fr_mctx_download(m, mean_rgb, rgb8);
  fr_mctx_free(m);
  return rc;
}

int fr_selftest_ops(int device, int op, const float* a, const float* b, uint32_t n, float* out) {
  if (!a || !b || !out) return set_error(FR_EARG, "fr_selftest_ops: null buffer");
  SET_DEVICE(device);
  float *da = nullptr, *db = nullptr, *dout = nullptr;
  const size_t bytes = (n ? n : 1) * sizeof(float);
  HIPCHK(hipMalloc(&da, bytes));
  HIPCHK(hipMalloc(&db, bytes));
  HIPCHK(hipMalloc(&dout, bytes));
  HIPCHK(hipMemcpy(da, a, n * sizeof(float), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(db, b, n * sizeof(float), hipMemcpyHostToDevice));
  if (n) hipLaunchKernelGGL(ops_kernel, dim3((n + 255) / 256), dim3(256), 0, 0, op, da, db, n, dout);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(out, dout, n * sizeof(float), hipMemcpyDeviceToHost));
  HIPCHK(hipFree(da));
  HIPCHK(hipFree(db));
  HIPCHK(hipFree(dout));
  return FR_OK;
}

int fr_selftest_rng(int device, uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, uint32_t* out) {
  if (!out) return set_error(FR_EARG, "fr_selftest_rng: null buffer");
  SET_DEVICE(device);
  uint32_t* d = nullptr;
  HIPCHK(hipMalloc(&d, (n ? n : 1) * sizeof(uint32_t)));
  hipLaunchKernelGGL(rng_kernel, dim3(1), dim3(64), 0, 0, seed, pixel, sample, n, d);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(out, d, n * sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIPCHK(hipFree(d));
  return FR_OK;
}

/* Diagnostic: exhaustive recip_nr check over [base, base + count) bit patterns;
   bad[256] / first[256] per exponent field (first = 0xFFFFFFFF when none). */
int fr_selftest_recip(int device, uint64_t base, uint64_t count, uint64_t* bad, uint32_t* first) {
  if (!bad || !first || base + count > (1ull << 32)) return set_error(FR_EARG, "fr_selftest_recip: bad arguments");
  SET_DEVICE(device);
  unsigned long long* dbad = nullptr;
  uint32_t* dfirst = nullptr;
  HIPCHK(hipMalloc(&dbad, 256 * sizeof(unsigned long long)));
  HIPCHK(hipMalloc(&dfirst, 256 * sizeof(uint32_t)));
  HIPCHK(hipMemset(dbad, 0, 256 * sizeof(unsigned long long)));
  HIPCHK(hipMemset(dfirst, 0xFF, 256 * sizeof(uint32_t)));
  if (count) hipLaunchKernelGGL(recip_check_kernel, dim3(8192), dim3(256), 0, 0, base, count, dbad, dfirst);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(bad, dbad, 256 * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(first, dfirst, 256 * sizeof(uint32_t), hipMemcpyDeviceToHost));
  HIPCHK(hipFree(dbad));
  HIPCHK(hipFree(dfirst));
  return FR_OK;
}

/* Diagnostic: div_rn against the IEEE division for every a mantissa and the b mantissas
   [b_base, b_base + b_count) (both operands in [1, 2)); *bad = differing pairs, *first =
   the least (b mantissa << 23 | a mantissa) among them (all ones when none). */
int fr_selftest_div(int device, uint32_t b_base, uint32_t b_count, uint64_t* bad, uint64_t* first) {
  if (!bad || !first || static_cast<uint64_t>(b_base) + b_count > (1ull << 23))
    return set_error(FR_EARG, "fr_selftest_div: bad arguments");
  SET_DEVICE(device);
  unsigned long long* d = nullptr;
  HIPCHK(hipMalloc(&d, 2 * sizeof(unsigned long long)));
  HIPCHK(hipMemset(d, 0, sizeof(unsigned long long)));
  HIPCHK(hipMemset(d + 1, 0xFF, sizeof(unsigned long long)));
  const uint32_t chunk = 512;  // b values per launch (2^32 pairs, a few ms)
  for (uint32_t k = 0; k < b_count; k += chunk) {
    hipLaunchKernelGGL(div_check_kernel, dim3((1u << 21) / 256), dim3(256), 0, 0, b_base + k,
                       min(chunk, b_count - k), d, d + 1);
    HIPCHK(hipGetLastError());
  }
  unsigned long long h[2];
  HIPCHK(hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost));
  HIPCHK(hipFree(d));
  *bad = h[0];
  *first = h[1];
  return FR_OK;
}

}  // extern "C"
