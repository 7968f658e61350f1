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
#ifdef FR_DIAG
// rejection-loop trip counters (wave trips via first active lane, lane tries)
__device__ unsigned long long g_fr_diag_lens[2];
__device__ unsigned long long g_fr_diag_rus[2];
#define FR_DIAG_TRY(arr)                                                           \
  do {                                                                             \
    const unsigned long long m_ = __ballot(1);                                     \
    if ((threadIdx.x & 63u) == static_cast<uint32_t>(__ffsll(m_) - 1)) {             \
      atomicAdd(&arr[0], 1ull);                                                    \
      atomicAdd(&arr[1], static_cast<unsigned long long>(__popcll(m_)));           \
    }                                                                              \
  } while (0)
// per-wave start/end (s_memrealtime, 100 MHz) for the residency-over-time profile
__device__ unsigned long long g_fr_wave_times[2 * 65536];
__device__ unsigned long long g_fr_wave_drain[65536];  // first drained claim of the wave
// segments traced per (sample block, tile) batch of 64 items: index item >> 6 (< 2^20 kept)
__device__ unsigned int g_fr_tb_cost[1u << 20];
// per wave: iterations at its first drained claim and at its end
__device__ unsigned int g_fr_wave_iters[2 * 65536];
// every 64th wave: the time of each of its first 1024 loop iterations (100 MHz)
__device__ unsigned long long g_fr_iter_times[1024 * 1024];
#define FR_LENS_TRY() FR_DIAG_TRY(g_fr_diag_lens)
#define FR_RUS_TRY() FR_DIAG_TRY(g_fr_diag_rus)
#endif
#include "rt_core.h"

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

constexpr uint32_t kBlock = 256;      // 4 waves, one 8x8 pixel tile each
constexpr uint32_t kStripRows = 8;    // rows per shard strip == tile height
constexpr uint32_t kMaxDepth = 64;    // LDS stack bound (64 KB per workgroup)
constexpr uint32_t kMaxWgPerCu = 8;   // 2048 threads per CU / kBlock: the persistent grid's cap
#ifndef FR_KREJ
#define FR_KREJ 4  // rejection loop: lanes left to the next iteration (tuning only, results unchanged)
#endif
// ... for the 8-B-record kernels (scenes of <= 15 primitives, the headline's): measured
// C3 trace 20.81 -> 20.69 ms at 6 (7 and 8 the same within noise); 6 on the other kernels
// cost C2 +1.7 % and a 10k-sphere BVH frame +1.2 %, so they keep FR_KREJ
#ifndef FR_KREJ_NIB
#define FR_KREJ_NIB 6
#endif
#ifndef FR_CLAIM_MIN
#define FR_CLAIM_MIN 1  // lanes that must wait for an item before the wave claims (tuning only)
#endif
// ... for the 8-B-record kernels (the headline's): C3 18.50 -> 18.28 ms at 2 (18.31 at 4, 18.46
// at 6); 4 on every kernel cost C2 +2 %, so the others keep FR_CLAIM_MIN
#ifndef FR_CLAIM_MIN_NIB
#define FR_CLAIM_MIN_NIB 2
#endif
#ifndef FR_NUM_SGPR
#define FR_NUM_SGPR 96
#endif
constexpr uint32_t kSmallDepth = 8;
// Deferred unwind (DEFER kernels: depth <= 8, <= kDeferMaxPrims primitives, no BVH, not
// render_mt): a path's sample slot holds the record {t, winners 0-3, winners 4-7} instead
// of its colour: t = the sky blend parameter 0.5 (unit(d).y + 1) of the escaping ray, or
// kDeferAbsorbed (-1, which no t in [0, 1] or NaN equals) for a path that returns 0; the
// winners as u8 primitive indices, kDeferUnit on empty levels. sum_kernel rebuilds
// a0 * (a1 * (... * term)) from it in the same order, at full SIMD width instead of in the
// few lanes whose paths end in a given iteration.
constexpr uint32_t kDeferMaxPrims = 254;
constexpr uint32_t kDeferUnit = 255;
constexpr uint32_t kDeferAbsorbed = 0xBF800000u;  // -1.0f
constexpr uint32_t KF_DEFER = 1u << 31;            // internal KParams.flags bit: records, not colours
constexpr uint32_t KF_STAGE = 1u << 30;            // internal: BVH kernel stages its samples in LDS
// Scenes of <= kNibbleMaxPrims primitives (the headline scene_08 has 6) keep the winners
// as 4-bit entries in one register instead of an LDS stack (15 = empty level) and store
// 8-B records {t, winners}: 2 words per sample instead of 3 (KF_NIBBLE, DEFER == 2).
constexpr uint32_t kNibbleMaxPrims = 15;
constexpr uint32_t kNibbleUnit = 15;
constexpr uint32_t KF_NIBBLE = 1u << 29;           // internal: 8-B deferred records
constexpr uint32_t KF_DIFFUSE = 1u << 28;          // internal: no metal/dielectric (trace_kernel MAT = 1)
#ifndef FR_BLOCK_SAMPLES
#define FR_BLOCK_SAMPLES 16  // RNG contract: one stream per 16-sample block (oracle.cpp agrees)
#endif
constexpr uint32_t kBlockSamples = FR_BLOCK_SAMPLES;  // samples per RNG stream (numerics contract)
// The last block of a pixel with more than one block is split into sub-blocks of
// kFineSamples samples, each its own stream (key kFineKey | s / kFineSamples): the queue
// ends with short items, so the drain after the last claim is short.
// (Splitting the last 2, 3 or 4 blocks measured 0.9-2.7 % slower at 1 GPU for 1-2 % at
// shard 0 of 8; one queue head per XCD, with stealing, 1.4 % slower.)
#ifndef FR_FINE_SAMPLES
#define FR_FINE_SAMPLES 4
#endif
constexpr uint32_t kFineSamples = FR_FINE_SAMPLES;
constexpr uint32_t kFineSub = kBlockSamples / kFineSamples;  // sub-blocks per block
constexpr uint32_t kFineKey = 0x80000000u;
static_assert(kFineSamples >= 1 && kBlockSamples % kFineSamples == 0 && kFineSub <= 4,
              "sub-block index packs into 2 bits of the claim's block word");
// work items reserved per step of the global counter: one tile of one sample block,
// seeded by the wave's 64 lanes at once (trace_kernel's claim step)
constexpr uint32_t kBatch = 64;

// ABI layout, mirrored by ctypes (forma_rt.py) and the Rust binding
static_assert(sizeof(fr_prim) == 88, "fr_prim layout");
static_assert(sizeof(fr_camera) == 104, "fr_camera layout");
static_assert(sizeof(fr_params) == 40, "fr_params layout");
static_assert(sizeof(fr_stats) == 72, "fr_stats layout");

struct DeviceCopy {
  int device = -1;
  uint64_t version = 0;
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
  bool att_nonneg = true;  // every attenuation component finite and >= +0 (no -0)
  bool diffuse = true;     // no metal or dielectric scatter class (trace_kernel MAT = 1)
};

struct KScene {
  // one 64-B record per primitive (g0..g3; kind in the bits of g3.w): one scalar
  // load brings a primitive into SGPRs in the closest-hit loop
  const float4* __restrict__ rec;
  const float4* __restrict__ mat;   // colour rgb, fuzz
  const uint32_t* __restrict__ cls; // effective ScatterClass
  const float4* __restrict__ att;   // attenuation rgb (colour, or 1 for light)
  const float4* __restrict__ bvh;   // BVH nodes, four float4 each (bvh.h)
  const uint32_t* __restrict__ bvh_order;  // primitive index of each leaf slot
  const float4* __restrict__ lrec;  // the primitives' records in leaf-slot order
  const uint4* __restrict__ segs;   // BvhSegment list: runs (one tree each) and planes, in list order
  // kind runs of the list (KS_ANY in-order loop): {kind, first, end, 0} for each maximal run
  // of consecutive primitives of one kind, in list order
  const uint4* __restrict__ runs;
  uint32_t n_runs;
  uint32_t n;
  uint32_t n_segs;                  // segment count (0: no BVH)
  uint32_t att_nonneg;              // every attenuation component finite and >= +0
  float reach;                      // BVH node cull is conservative for max|o_k| <= reach (bvh.h)
};

struct KParams {
  uint32_t W, H, spp, max_depth;
  uint64_t seed;
  uint32_t shard_index, shard_count, tiles_per_row, n_tiles, flags;
  uint32_t P;         // pixel slots of the shard: n_tiles x 64, tile order
  uint32_t b0, nb;    // this pass renders sample blocks [b0, b0 + nb)
  uint32_t n_items;   // nb x P work items (pixel slot, block); < 2^32 per pass
  uint32_t tiles_magic, tiles_shift;  // x / n_tiles = fastdiv(x, tiles_magic, tiles_shift)
  float rW, rH;                       // RN(1 / W), RN(1 / H) (host IEEE division)
  uint32_t row_magic, row_shift;      // x / tiles_per_row = fastdiv(x, row_magic, row_shift)
  uint32_t band_h;                    // FR_FLAG_MT_BANDS: rows per band, H / 4 (tracer.rs:87)
  uint32_t ks;          // sample slots per work item in the sample buffer: min(spp, kBlockSamples)
  // items handed out without the queue: wave w of the grid starts on batch w (one batch
  // per wave, n_static = waves x 64); the queue counts from n_static
  uint32_t n_static;
  // items [n_coarse, n_items) are the sub-blocks of block b_fine (the pixels' last block,
  // when spp > kBlockSamples and this pass holds it): item = n_coarse + k * P + q for
  // sub-block k; n_coarse = n_items when the pass has none
  uint32_t n_coarse, b_fine;
};

// Unsigned 32-bit division by the invariant n_tiles: q = (t + ((x - t) >> s1)) >> s2 with
// t = mulhi(x, m), l = ceil(log2 d), m = floor(2^32 (2^l - d) / d) + 1, s1 = min(l, 1),
// s2 = max(l - 1, 0) (Granlund-Montgomery; d = 1 gives m = 1, q = x). tests/test_fastdiv.py.
__host__ __device__ __forceinline__ uint32_t fastdiv(uint32_t x, uint32_t m, uint32_t shifts) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t t = __umulhi(x, m);
#else
  const uint32_t t = static_cast<uint32_t>((static_cast<uint64_t>(x) * m) >> 32);
#endif
  return (t + ((x - t) >> (shifts & 1u))) >> (shifts >> 1);
}

static void fastdiv_magic(uint32_t d, uint32_t& m, uint32_t& shifts) {
  if (d < 1) d = 1;
  const uint32_t l = d == 1 ? 0u : 32u - static_cast<uint32_t>(__builtin_clz(d - 1));
  m = static_cast<uint32_t>(((static_cast<uint64_t>(1) << 32) * ((static_cast<uint64_t>(1) << l) - d)) / d + 1);
  shifts = (l < 1 ? l : 1u) | ((l > 0 ? l - 1 : 0u) << 1);
}

// Work buffers of one render pass.
struct KWork {
  uint32_t* queue;            // next unclaimed item (zeroed before the pass)
  // per-sample colours or deferred records, item-major: sample s of item (b, q) at
  // [(item * ks + s - 16 b)] x WPS words (3, or 2 for 8-B records), item = (b - b0) * P + q,
  // so one item's samples are contiguous (192 or 128 B at ks = 16)
  float* samples;
  unsigned long long* counters;  // [0] segments, [1] hits, [2] scatters (reduce_counters)
  // per-wave partial counters, [wave][3], stored by every wave of the grid and summed
  // into counters by reduce_counters after the launch
  unsigned long long* wave_counters;
};

// camera.rs fields the ray generator reads: position, lower_left_corner,
// horizontal, vertical, u, v (named b* here), lens_radius
struct KCam {
  float px, py, pz, lx, ly, lz, hx, hy, hz, vx, vy, vz, ux, uy, uz, bx, by, bz, lens;
};

struct KArgs {
  KScene sc;
  KCam cam;
  KParams kp;
  KWork kw;
};

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

__device__ __forceinline__ V3 xyz(float4 a) { return V3{a.x, a.y, a.z}; }

// The scene is read-only for the kernel's lifetime: reading it through the constant
// address space lets the compiler use scalar loads even though the kernel stores to
// global memory inside the same loop.
typedef __attribute__((address_space(4))) const float cfloat;
struct RecRef {  // the 4 float4 of one primitive record, read through addrspace(4)
  cfloat* p;
  __device__ __forceinline__ float4 operator[](int k) const {
    return make_float4(p[4 * k], p[4 * k + 1], p[4 * k + 2], p[4 * k + 3]);
  }
};
__device__ __forceinline__ RecRef rec_at(const float4* base, uint32_t i) {
  return RecRef{(cfloat*)(reinterpret_cast<uintptr_t>(base)) + 16u * i};
}

// Raw buffer loads (SGPR resource over a uniform base pointer). Used where an LDS and a
// global read of the same value sit on two sides of a uniform branch: a buffer load
// cannot be merged with the LDS read into one generic (flat) load.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7FFFFFFF, 0x00020000);
}
__device__ __forceinline__ float4 buf_load4(const void* base, uint32_t byte_off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(buf_rsrc(base), byte_off, 0, 0));
}
__device__ __forceinline__ uint32_t buf_load1(const void* base, uint32_t byte_off) {
  return __builtin_amdgcn_raw_buffer_load_b32(buf_rsrc(base), byte_off, 0, 0);
}

constexpr uint32_t kAttLds = 1024;  // attenuation/class entries staged in LDS (16 B each)
constexpr uint32_t kRecLds = 64;    // whole 64-B records staged in LDS for small scenes
// Sample colours a lane stages in LDS before storing them to the (item-major) sample
// buffer: 4 x 12 B = three 16-B stores per 4 samples (4 x 8 B = two, for 8-B records)
// instead of four scattered stores, which L2 wrote back as partial lines (3.5x WRITE_SIZE).
// The BVH kernels stage 2 samples when their LDS allows (below).
#ifndef FR_STAGE
#define FR_STAGE 4  // 1 or 4 (A/B builds)
#endif
// The BVH kernels stage 2 samples when the 6 KB this adds to their LDS (which holds the
// traversal stack) keeps their resident workgroups per CU (KF_STAGE, decided at launch):
// C5 66.8 -> 64.3 ms; on scenes whose LDS tables fill the CU it would cost a workgroup.
#ifndef FR_BVH_STAGE
#define FR_BVH_STAGE 2
#endif
__host__ __device__ constexpr uint32_t stage_samples(bool bvh) { return bvh ? FR_BVH_STAGE : FR_STAGE; }
// a sub-block starts on a staging group: the group's store covers only its own samples
static_assert(kFineSamples % FR_STAGE == 0, "sub-blocks hold whole staging groups");

// FR_DIAG builds count, per phase, wave-level trips (one per SIMT pass of the wave)
// and lane-level work, to measure SIMT efficiency. Never enabled in the product.
#ifdef FR_DIAG
enum { DG_ITER, DG_REGEN_W, DG_REGEN_L, DG_LENS_W, DG_LENS_L, DG_RUS_W, DG_RUS_L, DG_END_W, DG_END_L,
       DG_UNW_W, DG_UNW_L, DG_HIT_W, DG_NODE_W, DG_NODE_L, DG_LEAF_W, DG_LEAF_L, DG_N };
#define DIAG_WAVE(slot)                                                         \
  do {                                                                          \
    const unsigned long long m_ = __ballot(1);                                  \
    if (lane == static_cast<uint32_t>(__ffsll(m_) - 1)) atomicAdd(&dg[slot], 1u); \
  } while (0)
#define DIAG_LANE(slot)                                                         \
  do {                                                                          \
    const unsigned long long m_ = __ballot(1);                                  \
    if (lane == static_cast<uint32_t>(__ffsll(m_) - 1))                         \
      atomicAdd(&dg[slot], static_cast<uint32_t>(__popcll(m_)));                \
  } while (0)
#else
#define DIAG_WAVE(slot) do {} while (0)
#define DIAG_LANE(slot) do {} while (0)
#endif

// FR_PROF builds read the shader clock (s_memtime, wave-uniform) at the section
// boundaries of the lane loop and add each wave's cycles per section into
// counters[20 + k]: wall-clock residency by section. Never enabled in the product.
#ifdef FR_PROF
enum { PF_CLAIM, PF_REJ, PF_HIT, PF_SHADE, PF_END, PF_N };
#define PROF_MARK(k)                                       \
  do {                                                     \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();      \
    pf_acc[k] += t_ - pf_t;                                \
    pf_t = t_;                                             \
  } while (0)
#else
#define PROF_MARK(k) do {} while (0)
#endif

// HAS_PLANE: planes may leave the shared record's t/p stale (plane.rs:27-29), so
// the last written t is tracked separately from the winner's.
// (two 32-bit popcounts: a 64-bit one leaves a 64-bit count whose compare the SALU
// cannot do, and the compiler moved it to the VALU)
__device__ __forceinline__ uint32_t lanes_set(bool b) {
  const unsigned long long m = __ballot(b);
  return static_cast<uint32_t>(__builtin_popcount(static_cast<uint32_t>(m)) +
                               __builtin_popcount(static_cast<uint32_t>(m >> 32)));
}

// Pixel slot q of a shard -> image coordinates. Slots run tile by tile (8x8 pixels,
// tiles left to right within an 8-row strip, the shard's strips top to bottom); slots
// past the image edge are invalid.
__device__ __forceinline__ bool slot_xy(const KParams& kp, uint32_t q, uint32_t& x, uint32_t& y) {
  const uint32_t tile = q >> 6, l = q & 63u;
  const uint32_t ls = fastdiv(tile, kp.row_magic, kp.row_shift);  // tile / tiles_per_row
  const uint32_t tc = tile - ls * kp.tiles_per_row;
  const uint32_t strip = kp.shard_index + ls * kp.shard_count;
  x = tc * 8u + (l & 7u);
  y = strip * kStripRows + (l >> 3);
  return x < kp.W && y < kp.H;
}

// Work item -> (block word bw, pixel slot q, image x, y); false for a slot past the image
// edge. item = (b - b0) * P + q with P = 64 * n_tiles (split via the tile-block index),
// or n_coarse + k * P + q for sub-block k of block b_fine. bw = b for a whole block,
// b | kFineKey | k << 28 for a sub-block (b < 2^28: spp < 2^32).
__device__ __forceinline__ bool item_xy(const KParams& kp, uint32_t item, uint32_t& bw, uint32_t& q, uint32_t& x,
                                        uint32_t& y) {
  const bool fine = item >= kp.n_coarse;
  const uint32_t tb = (fine ? item - kp.n_coarse : item) >> 6;  // n_coarse is a multiple of 64
  const uint32_t bl = fastdiv(tb, kp.tiles_magic, kp.tiles_shift);
  bw = fine ? (kp.b_fine | kFineKey | (bl << 28)) : kp.b0 + bl;
  q = ((tb - bl * kp.n_tiles) << 6) | (item & 63u);
  return slot_xy(kp, q, x, y);
}

// RNG stream key of a block word: the block index, or kFineKey | s / kFineSamples for a
// sub-block starting at sample s (oracle.cpp stream_key agrees)
__host__ __device__ __forceinline__ uint32_t stream_key(uint32_t bw) {
  return (bw & kFineKey) ? (kFineKey | ((bw & 0x0FFFFFFFu) * kFineSub + ((bw >> 28) & 3u))) : bw;
}

// Persistent path-tracing kernel. Work item = (pixel slot q, sample block b): the
// kBlockSamples samples [16b, 16b + 16) of one pixel, drawn in order from the RNG
// stream (seed, pixel, b). Each sample's colour goes to kw.samples; sum_kernel then
// adds every pixel's samples in sample order, exactly as save_image's
// `col = col + get_color(...)` (tracer.rs:170-175). Items are independent, so lanes
// never wait for one another's pixels: a wave claims 64 items (one tile, one block)
// per global atomic and hands them to its free lanes (ballot + mbcnt).
//
// Per iteration of the lane loop:
//   0. lanes without an item claim one;
//   1. one merged rejection loop serves both random_in_unit_circle (lens sample of a
//      new camera ray, utility.rs:4-13) and random_in_unit_sphere (scatter,
//      utility.rs:15-25): a circle try is a sphere try without the third draw, and
//      dot(p,p) = (px*px + py*py) + 0 is the same value. It stops once at most KREJ
//      lanes still reject; those keep their RNG state and go on next iteration (their
//      draws stay in stream order, so results do not depend on KREJ);
//   2. closest hit + shading for lanes holding a ray;
//   3. path end: unwind the attenuations, store the sample colour, next sample.
// MAXD > 0: max_depth <= MAXD is known at compile time; the stack holds u16 primitive
// indices (n < 65536) and is unwound by an unrolled, predicated sequence.
// MAXD == 0: any max_depth, u32 indices, a loop.
// KS: KS_AABB / KS_SPHERE when every primitive has that kind (no per-primitive kind
// switch), else KS_ANY.
enum { KS_ANY = 0, KS_AABB = 1, KS_SPHERE = 2 };

// f(integral_constant<I>) for I = I0, I0 + 1, ... while I < n (n <= N), unrolled
template <uint32_t I, uint32_t N, class F>
__device__ __forceinline__ void unroll_below(uint32_t n, F& f) {
  if constexpr (I < N) {
    if (I < n) {
      f(std::integral_constant<uint32_t, I>{});
      unroll_below<I + 1u, N>(n, f);
    }
  }
}

// amdgpu_num_sgpr caps the scalar registers (MI355X_MICROARCH.md "Residency and
// cooperative launch": <= 80 SGPRs admit 8 workgroups of 256 threads per CU, 82-96
// admit 7). Measured on scene_08: 96 beats 80 (fewer SGPR spills) and 102.
// MAT = 1: no metal or dielectric primitive (every scatter is lambertian: lambertian, light,
// or none for stubs): the shading step drops those branches (the headline scene's case).
template <int KS, bool HAS_PLANE, int KREJ, int MAXD, bool BVH, bool MT, int DEFER, int MAT = 0>
// Waves per SIMD the kernels ask for: the list-loop kernels at least 7 (<= 72 VGPRs), the
// BVH kernels at least 6 (<= 80); without the request the general (KS_ANY) and BVH
// kernels settle at 83-94 VGPRs, 5 waves. Measured (tools/ab_bench.py): 7 for the list
// kernels (scene_01 C2 37.9 -> 36.0 ms, a few VGPRs spilled to scratch), 6 for the BVH
// ones (7 or 8 spill more: C5 +2-10 %, scene_06 +12-20 %). FR_MIN_WAVES=n forces n.
#ifdef FR_MIN_WAVES
#define FR_OCC_ATTR __attribute__((amdgpu_waves_per_eu(FR_MIN_WAVES)))
#else
#ifndef FR_NIB_WAVES
// the 8-B-record (headline) kernel at 8 waves: with FR_KREJ_NIB = 6, C3 trace 20.67 ->
// 20.49 ms and shard 0/4 -0.6 % (shard 0/8 +0.3 %); at KREJ 4 it had measured -0.3 % / +1.1 %
#define FR_NIB_WAVES 8
#endif
#ifndef FR_DIFF12_WAVES
#define FR_DIFF12_WAVES 7  // diffuse-only 12-B-record kernels (A/B knob)
#endif
#define FR_OCC_ATTR \
  __attribute__((amdgpu_waves_per_eu(BVH ? 6 : DEFER == 2 ? FR_NIB_WAVES : (DEFER == 1 && MAT == 1) ? FR_DIFF12_WAVES : 7)))
#endif
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_num_sgpr(FR_NUM_SGPR))) FR_OCC_ATTR void trace_kernel(
    KArgs args) {
  // one by-value struct: the kernarg segment holds it at offset 0 (the camera is read
  // back from there in the lens step)
  const KScene& sc = args.sc;
  const KParams& kp = args.kp;
  const KWork& kw = args.kw;
  // LDS: [n_att + 1 x (attenuation rgb, scatter class bits)][n_rec x 64-B record]
  //      [stack: MAXD ? kBlock x MAXD u16 (lane-major) : max_depth x kBlock u32]
  // Entry n of the attenuations is (1, 1, 1): the depth-8 stack's empty levels hold n.
  // Staging the winner's data keeps per-lane global gathers off the shading path.
  // [STG > 1: kBlock x STG staged sample colours (12 B each), lane-major] in front.
  extern __shared__ uint32_t lds[];
  constexpr uint32_t STG = stage_samples(BVH);
  constexpr bool NIB = DEFER == 2;             // 8-B records, winners in a register
  constexpr bool DIFFUSE = MAT == 1;           // lambertian scatters only
  constexpr uint32_t WPS = NIB ? 2u : 3u;      // words per sample in the buffer
  // list kernels always stage; BVH kernels when the launch gave them the LDS (KF_STAGE)
  const bool staged = STG > 1 && (!BVH || (kp.flags & KF_STAGE) != 0u);
  float* stage = reinterpret_cast<float*>(lds) + threadIdx.x * (WPS * STG);
  // DEFER kernels (<= kDeferMaxPrims primitives) always hold the attenuations in LDS, and
  // the 8-B-record kernels (<= kNibbleMaxPrims) the records too: compile-time facts there,
  // so their global-load fallbacks are not compiled
  constexpr bool ATT_LDS = DEFER != 0, REC_LDS = NIB;
  static_assert(kDeferMaxPrims <= kAttLds && kNibbleMaxPrims <= kRecLds, "LDS staging bounds");
  const uint32_t n_att = ATT_LDS || sc.n <= kAttLds ? sc.n : 0u;
  const uint32_t n_att_st = n_att ? n_att + 1u : 0u;  // with the unit entry
  const uint32_t n_rec = REC_LDS || sc.n <= kRecLds ? sc.n : 0u;
  float4* att_lds = reinterpret_cast<float4*>(lds + (staged ? kBlock * WPS * STG : 0u));
  float4* rec_lds = att_lds + n_att_st;
  uint32_t* stack = reinterpret_cast<uint32_t*>(rec_lds + 4u * n_rec);
  uint16_t* hstack = reinterpret_cast<uint16_t*>(stack);
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
  static_assert(MAXD == 0 || MAXD == 8, "the u16 stack is one 16-B row per lane");
  static_assert(!DEFER || (MAXD == 8 && !BVH && !MT), "deferred unwind: depth <= 8 list kernels");
  uint2* drow = reinterpret_cast<uint2*>(stack) + tid;  // DEFER: this lane's 8 u8 levels
  uint8_t* bstack = reinterpret_cast<uint8_t*>(stack);
  uint4* hrow = reinterpret_cast<uint4*>(stack) + tid;  // this lane's MAXD = 8 levels
  // BVH traversal stack, after the unwind stack: kBvhStack x kBlock u32 (level-major)
  uint32_t* tstack = stack + (MAXD ? (MAXD * kBlock) / 2u : (kp.max_depth ? kp.max_depth : 1u) * kBlock);
  // MAXD > 0 stack entries: with the attenuations in LDS, the entry's byte offset in
  // att_lds (n_att <= kAttLds, so < 2^16), read by the unwind without index arithmetic;
  // otherwise the primitive index
  const uint32_t ent_shift = n_att ? 4u : 0u;
  const uint32_t unit_ent = sc.n << ent_shift;
  const uint32_t unit2 = unit_ent | (unit_ent << 16);  // two empty levels
  if (DEFER == 1)
    *drow = make_uint2(~0u, ~0u);
  else if (!DEFER && MAXD > 0)
    *hrow = make_uint4(unit2, unit2, unit2, unit2);
  for (uint32_t i = tid; i < n_att_st; i += kBlock) {
    const float4 a = sc.att[i];
    att_lds[i] = make_float4(a.x, a.y, a.z, __uint_as_float(i < n_att ? sc.cls[i] : 0u));
  }
  for (uint32_t i = tid; i < 4u * n_rec; i += kBlock) rec_lds[i] = sc.rec[i];
#ifdef FR_DIAG
  __shared__ uint32_t dg[DG_N];
  if (tid < DG_N) dg[tid] = 0;
  const uint32_t gw = blockIdx.x * (kBlock / 64u) + (tid >> 6);
  if (lane == 0 && gw < 65536) {
    g_fr_wave_times[2 * gw] = __builtin_amdgcn_s_memrealtime();
    g_fr_wave_drain[gw] = ~0ull;
  }
#endif
  __syncthreads();


  const float fW = static_cast<float>(kp.W), fH = static_cast<float>(kp.H);

  enum : uint32_t { NEED_NONE = 0, NEED_LENS = 1, NEED_SPHERE = 2 };
  uint32_t depth = 0;
  uint32_t wnib = ~0u;  // NIB: the winners, level k in bits 4k..4k+3 (15: empty)
  // stack push at level `depth` of the scatter winner
  auto push = [&](uint32_t pi) {
    if (NIB)
      wnib ^= (pi ^ kNibbleUnit) << (4u * depth);
    else if (DEFER)
      bstack[tid * 8u + depth] = static_cast<uint8_t>(pi);
    else if (MAXD > 0)
      hstack[tid * MAXD + depth] = static_cast<uint16_t>(pi << ent_shift);
    else
      stack[depth * kBlock + tid] = pi;
  };

  // the ray; while a lens sample is pending d.xy = (u, v); while a scatter sample is
  // pending o = hit point and d = scatter base ((p + n), or reflect(unit(d), n) for metal)
  V3 o{0.0f, 0.0f, 0.0f}, d{0.0f, 0.0f, 1.0f};
  V3 sn{0.0f, 0.0f, 0.0f};  // metal: normal
  float sfuzz = 0.0f, fx = 0.0f, fy = 0.0f, vofs = 0.0f;
  bool smetal = false;
  uint32_t sbest = 0, s = 0, s_end = 0, nseg = 0, nhit = 0, nscat = 0;
  uint32_t jj = 0;           // sample index within the item's block
#ifdef FR_DIAG
  uint32_t diag_tb = 0, diag_seg0 = 0;  // the item's batch index, segments at its claim
  uint32_t diag_iter = 0;               // loop iterations of this wave
#endif
  float* out = kw.samples;   // the item's first sample slot (item-major buffer)
  Rng rng{0u, 0u, 0u, 0u};
  bool active = true, need_item = true, need_jit = false, have_ray = false;
  uint32_t need = NEED_NONE;

#ifdef FR_PROF
  uint64_t pf_acc[PF_N] = {0, 0, 0, 0, 0};
  uint64_t pf_t = __builtin_amdgcn_s_memtime();
#endif
  // the wave's claimed item batch [q_next, q_end): wave-uniform, updated only under
  // the uniform branch below, so it lives in scalar registers
  uint32_t q_next = 0, q_end = 0;
  // Stream starts of the wave's batch: lane k holds item (batch base + k)'s. The whole
  // wave seeds a batch when it reserves one, so rng_seed (16 quarter-rate 32-bit
  // multiplies) runs once per 64 items at full width instead of in every iteration in
  // which a lane or two claim; a claiming lane fetches its stream by a lane permute.
  Rng held{0u, 0u, 0u, 0u};
  // ... and the same slot's pixel (x | y << 16, all ones past the image edge) and sample
  // block, so a claiming lane fetches those by permute too instead of dividing the item
  uint32_t held_xy = 0xFFFFFFFFu, held_b = 0u;
  // A wave's first batch is its own (wave w of the grid: batch w), seeded here: 7168
  // first claims at once on one counter would queue for ~80 us (about 88 returning
  // atomics per us on one word, MI355X_MICROARCH.md "dequeue").
  {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(4))) const KArgs cargs_0;
    cargs_0* ap0 = (cargs_0*)(__builtin_amdgcn_kernarg_segment_ptr());
    asm volatile("" : "+s"(ap0));
    const KParams k0 = ap0->kp;
#else
    const KParams& k0 = kp;
#endif
    q_next = (blockIdx.x * (kBlock / 64u) + (tid >> 6)) * kBatch;
    q_end = q_next + kBatch;
    uint32_t bb, qq, xx, yy;
    const bool in_image = item_xy(k0, q_next + lane, bb, qq, xx, yy);
    held = rng_seed(k0.seed, yy * k0.W + xx, stream_key(bb));
    held_xy = in_image ? (xx | (yy << 16)) : 0xFFFFFFFFu;
    held_b = bb;
  }
  while (active) {
    DIAG_WAVE(DG_ITER);
#ifdef FR_DIAG
    if (lane == 0 && (gw & 63u) == 0 && (gw >> 6) < 1024u && diag_iter < 1024u)
      g_fr_iter_times[(gw >> 6) * 1024u + diag_iter] = __builtin_amdgcn_s_memrealtime();
    ++diag_iter;
#endif
    const unsigned long long m = __ballot(need_item);
    // Lanes whose item is done wait (idle) until FR_CLAIM_MIN of them need one, or until no
    // active lane has other work: the claim step (its lane permutes and item setup) then
    // runs for several lanes at once instead of in nearly every iteration for one or two.
    // Only when work starts changes, never what a sample computes (results bit-identical).
    constexpr uint32_t CLAIM_MIN = NIB ? FR_CLAIM_MIN_NIB : FR_CLAIM_MIN;
    if (m && (CLAIM_MIN <= 1 || lanes_set(need_item) >= CLAIM_MIN || m == __ballot(1))) {
      // 0. claim work items: the free lanes take consecutive items of the wave's batch;
      // when it runs out, the first free lane reserves the next batch of kBatch = 64
      // items (one tile of one sample block) globally. n <= 64, so one batch suffices.
      // (Prefetching the next item in batched refill passes measured slower.)
      const uint32_t n = static_cast<uint32_t>(__popcll(m));
      const uint32_t r = __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                                   __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
      const uint32_t next = __builtin_amdgcn_readfirstlane(q_next);
      const uint32_t avail = __builtin_amdgcn_readfirstlane(q_end) - next;
      uint32_t base = 0;
      const bool grab = n > avail;
      const int first = __ffsll(static_cast<long long>(m)) - 1;
      // The item's stream start, pixel and block, by lane permute from the lane that
      // seeded them: first from the current batch (claims r < avail), then, after a grab,
      // from the new batch (claims r >= avail). Every lane of the wave is active at both
      // permutes (a permute reads 0 from an inactive source): a lane retires only after
      // the queue has drained, and from then on no batch holds a valid item.
      int sl = static_cast<int>(((next + r) & (kBatch - 1u)) << 2);
      Rng st{static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(sl, static_cast<int>(held.s0))),
             static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(sl, static_cast<int>(held.s1))),
             static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(sl, static_cast<int>(held.s2))),
             static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(sl, static_cast<int>(held.s3)))};
      uint32_t xy = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(sl, static_cast<int>(held_xy)));
      uint32_t b = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(sl, static_cast<int>(held_b)));
      if (grab) {
        if (static_cast<int>(lane) == first) base = atomicAdd(kw.queue, kBatch);
        base = __builtin_amdgcn_readlane(base, first);
        // A slot past the image or the queue gets a stream that is never used.
#if defined(__HIP_DEVICE_COMPILE__)
        // the item split's parameters reloaded from the kernarg segment here (once per 64
        // items) rather than held in SGPRs across the loop, like the camera (step 1)
        typedef __attribute__((address_space(4))) const KArgs cargs_g;
        cargs_g* apg = (cargs_g*)(__builtin_amdgcn_kernarg_segment_ptr());
        asm volatile("" : "+s"(apg));
        const KParams kg = apg->kp;
#else
        const KParams& kg = kp;
#endif
        base += kg.n_static;  // past the waves' first batches
        q_end = base + kBatch;
        uint32_t bb, qq, xx, yy;
        const bool in_image = item_xy(kg, base + lane, bb, qq, xx, yy);
        held = rng_seed(kg.seed, yy * kg.W + xx, stream_key(bb));
        held_xy = in_image ? (xx | (yy << 16)) : 0xFFFFFFFFu;
        held_b = bb;
        // claims r >= avail take the new batch's slots r - avail (base is a multiple of 64)
        sl = static_cast<int>(((r - avail) & (kBatch - 1u)) << 2);
        const Rng st2{static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(sl, static_cast<int>(held.s0))),
                      static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(sl, static_cast<int>(held.s1))),
                      static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(sl, static_cast<int>(held.s2))),
                      static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(sl, static_cast<int>(held.s3)))};
        const uint32_t xy2 = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(sl, static_cast<int>(held_xy)));
        const uint32_t b2 = static_cast<uint32_t>(__builtin_amdgcn_ds_bpermute(sl, static_cast<int>(held_b)));
        if (r >= avail) {
          st = st2;
          xy = xy2;
          b = b2;
        }
      }
      q_next = grab ? base + (n - avail) : next + n;
      const uint32_t item = r < avail ? next + r : base + (r - avail);
      if (need_item && item >= kp.n_items) {
#ifdef FR_DIAG
        if (gw < 65536) {
          const unsigned long long now = __builtin_amdgcn_s_memrealtime();
          if (now < g_fr_wave_drain[gw]) {
            g_fr_wave_drain[gw] = now;
            g_fr_wave_iters[2 * gw] = diag_iter;
          }
        }
#endif
        active = false;  // queue drained
        continue;
      }
      if (need_item) {
        const uint32_t x = xy & 0xFFFFu, y = xy >> 16;
        bool ok = xy != 0xFFFFFFFFu;
        uint32_t yrow = kp.H - y;  // tracer.rs:171-172: v = ((H - y) + r) / H
        if (MT) {
          // render_mt (tracer.rs:86-103): band k from the top is thread t_id = 3 - k;
          // v = ((t_height - y_band) + r) / H + t_id * 0.25; rows past 4 * t_height unused
          const uint32_t k = kp.band_h ? y / kp.band_h : 4u;
          ok = ok && k < 4u;
          yrow = kp.band_h - (y - k * kp.band_h);
          vofs = static_cast<float>(3u - k) * 0.25f;
        }
        if (ok) {
          rng = st;  // this item's stream: rng_seed(seed, y * W + x, stream_key(b))
          // a sub-block k of block b_fine: samples [16 b + 4 k, +4) of the block's slot
          // (item - k * P in the buffer); a whole block: k = 0
          const uint32_t k = (b >> 28) & 3u;
          const bool fine = (b & kFineKey) != 0u;
          jj = k * kFineSamples;
          s = (b & 0x0FFFFFFFu) * kBlockSamples + jj;
          out = kw.samples + WPS * (static_cast<size_t>(item - k * kp.P) * kp.ks);
#ifdef FR_DIAG
          diag_tb = item >> 6;
          diag_seg0 = nseg;
#endif
          s_end = min(s + (fine ? kFineSamples : kBlockSamples), kp.spp);
          fx = static_cast<float>(x);
          fy = static_cast<float>(yrow);
          need_jit = true;
          need_item = false;
        }
      }
    }
    if (need_jit) {
      // a sample starts: jitter (tracer.rs:171-172), then its lens sample in step 1. One
      // place for the first sample of a block and the next sample of the same block, so
      // the wave runs it once per iteration
      const float r0 = rng_f32(rng);
      const float r1 = rng_f32(rng);
      d.x = div_rn(fx + r0, fW, kp.rW);  // (fx + r0) / fW, numerator +0 or in [2^-24, 2^32]
      d.y = div_rn(fy + r1, fH, kp.rH);
      if (MT) d.y = d.y + vofs;  // render_mt's band offset (tracer.rs:103)
      need = NEED_LENS;
      need_jit = false;
    }
    PROF_MARK(PF_CLAIM);
    bool ended = false;
    V3 term{0.0f, 0.0f, 0.0f};
    uint32_t tsky = kDeferAbsorbed;  // DEFER: the terminal as sky parameter bits
    if (need != NEED_NONE) {
      // 1. merged rejection loop
      float px = 0.0f, py = 0.0f, pz = 0.0f;
      bool acc = false;
      const bool sph = need == NEED_SPHERE;
      do {
        DIAG_WAVE(DG_LENS_W);
        DIAG_LANE(DG_LENS_L);
        if (!acc) {
          // the test in the 2^23-scaled domain (rng_signed_unit_scaled): same decisions
          px = rng_signed_unit_scaled(rng);
          py = rng_signed_unit_scaled(rng);
          if (sph) pz = rng_signed_unit_scaled(rng);  // a circle try keeps pz = 0
          acc = !(px * px + py * py + pz * pz >= kUnitBallScaled);
        }
      } while (lanes_set(!acc) > static_cast<uint32_t>(KREJ));
      if (acc) {
        px *= kSignedUnitScale;  // the accepted point, 2r - 1 per coordinate (exact)
        py *= kSignedUnitScale;
        pz *= kSignedUnitScale;
        if (!sph) {
          // Camera::get_ray (camera.rs:62-72)
#if !defined(FR_CAM_RESIDENT) && defined(__HIP_DEVICE_COMPILE__)
          // scalar loads of the camera from the kernarg segment, here, rather than 19
          // SGPRs held (and spilled) across the loop: the pointer is opaque to the
          // compiler, so the loads stay in this step
          typedef __attribute__((address_space(4))) const KArgs cargs;
          cargs* ap = (cargs*)(__builtin_amdgcn_kernarg_segment_ptr());
          asm volatile("" : "+s"(ap));
          const KCam cm = ap->cam;
#else
          const KCam& cm = args.cam;
#endif
          const V3 cpos{cm.px, cm.py, cm.pz}, cllc{cm.lx, cm.ly, cm.lz}, chor{cm.hx, cm.hy, cm.hz};
          const V3 cver{cm.vx, cm.vy, cm.vz}, cu{cm.ux, cm.uy, cm.uz}, cv{cm.bx, cm.by, cm.bz};
          const V3 rd = scl(cm.lens, V3{px, py, 0.0f});
          const V3 off = add(scl(rd.x, cu), scl(rd.y, cv));
          const float u = d.x, v = d.y;
          o = add(cpos, off);
          d = sub(sub(add(add(cllc, scl(u, chor)), scl(v, cver)), cpos), off);
          depth = 0;
          have_ray = true;
        } else {
          const V3 r{px, py, pz};
          bool ok = true;
          V3 dir;
          if (!DIFFUSE && smetal) {
            dir = add(d, scl(sfuzz, r));  // reflected + fuzz * rus
            ok = dot(dir, sn) > 0.0f;     // sphere.rs:104 / plane.rs:121
          } else {
            dir = sub(add(d, r), o);  // ((p + n) + rus) - p
          }
          if (ok) {
            push(sbest);
            ++depth;
            ++nscat;
            d = dir;
            have_ray = true;
          } else {
            ended = true;  // absorbed: get_color returns 0
          }
        }
        need = NEED_NONE;
      }
    }
    PROF_MARK(PF_REJ);
    if (have_ray) {
      // 2. closest hit over the list in order (tracer.rs:190-200): only the accepted t
      // of each test is needed here; the record is formed for the winner below.
      ++nseg;
      V3 inv{recip_nr(d.x), recip_nr(d.y), recip_nr(d.z)};
      // (non-short-circuit: one branch to the rare fallback instead of three nested ones)
      const int rok = static_cast<int>(recip_nr_ok(d.x)) & static_cast<int>(recip_nr_ok(d.y)) &
                      static_cast<int>(recip_nr_ok(d.z));
      if (!rok) inv = V3{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
      const float a_dd = dot(d, d);
#ifndef FR_SPHERE_IEEE
      const SphereSeg ssg = sphere_seg(a_dd);  // unused (removed) in kernels without spheres
#endif
      float closest = FLT_MAX, t_last = 0.0f;
      int best = -1;
      // The node cull is conservative only for origins within kBvhOriginReach scene
      // extents (bvh.h). A stale plane record (plane.rs:27-40) can put a scatter origin
      // p = o + t_stale d far outside: a wave holding such a lane (or a NaN origin) tests
      // the list in order instead, which the BVH walk equals bit for bit.
      bool list_walk = !BVH;
      if (BVH) {
        const float ao = fmax3_num(__builtin_fabsf(o.x), __builtin_fabsf(o.y), __builtin_fabsf(o.z));
        list_walk = __ballot(!(ao <= sc.reach)) != 0;
      }
      if (BVH && !list_walk) {
        // The list cut at its planes (bvh.h), walked in list order: each plane tested
        // where it stands, each run of other primitives through its own tree. A
        // primitive's candidate t does not depend on t_max, so a run's effect is the
        // least (t, index) of the run below `closest`: a primitive listed before the
        // current winner may take an exact tie, tested with t_max one ulp above
        // closest. Boxes are padded, so no primitive the list loop accepts is culled
        // (DESIGN.md §4.8). A lane steps into the nearer entered child and stacks the
        // other; lanes that reach a leaf wait for the wave's others, so leaves are
        // tested together.
        typedef __attribute__((address_space(4))) const uint32_t cu32;
        for (uint32_t sg = 0; sg < sc.n_segs; ++sg) {
          const cu32* sp = (cu32*)(reinterpret_cast<uintptr_t>(sc.segs)) + 4u * __builtin_amdgcn_readfirstlane(sg);
          if (HAS_PLANE && sp[0]) {
            const uint32_t i = sp[3];
            const RecRef r4 = rec_at(sc.rec, i);  // scalar loads
            float t = 0.0f;
            const int r = plane_test(xyz(r4[0]), xyz(r4[1]), xyz(r4[2]), o, d, 0.001f, closest, t);
            if (r) t_last = t;
            if (r == 2) {
              closest = t;
              best = static_cast<int>(i);
            }
            continue;
          }
          uint32_t ref = sp[1];
          uint32_t depth_s = 0;  // entries on this lane's traversal stack
          // node slabs as fma(lo, inv, -o inv): a cull only, covered by the padding for
          // origins within kBvhOriginReach scene extents (bvh.h; the host checks the camera).
          // The cull's reciprocal is clamped to +-2^100 (bvh.h kBvhInvClamp): an exact-zero
          // direction component (a lambertian bounce ((p + n) + r) - p at |p| ~ 5000 gives one
          // every few thousand scatters) has inv = +-inf, and fma(lo, inf, -(o inf)) is
          // inf - inf = NaN, which culled boxes the ray is inside. With the clamp, o inv is
          // finite and a slab that holds the ray's hit by the padding (>= 1e-4) stays
          // >= 1e-4 * 2^100 wide on that axis.
          const V3 invc{__builtin_amdgcn_fmed3f(inv.x, -kBvhInvClamp, kBvhInvClamp),
                        __builtin_amdgcn_fmed3f(inv.y, -kBvhInvClamp, kBvhInvClamp),
                        __builtin_amdgcn_fmed3f(inv.z, -kBvhInvClamp, kBvhInvClamp)};
          const V3 oinv{o.x * invc.x, o.y * invc.y, o.z * invc.z};
          while (ref != kBvhEnd) {
            while (ref < kBvhLeaf) {
              DIAG_WAVE(DG_NODE_W);
              DIAG_LANE(DG_NODE_L);
              // internal node: both children's boxes
              float4 na, nb, nc;
              uint4 nr;
              const uint32_t ref0 = __builtin_amdgcn_readfirstlane(ref);
              if (__ballot(ref != ref0) == 0) {
                // every walking lane is at the same node (coherent rays near the root):
                // scalar loads, which return sooner than the vector path
                const RecRef nd = rec_at(sc.bvh, ref0);
                na = nd[0];
                nb = nd[1];
                nc = nd[2];
                const float4 r = nd[3];
                nr = make_uint4(__float_as_uint(r.x), __float_as_uint(r.y), __float_as_uint(r.z), __float_as_uint(r.w));
              } else {
                na = sc.bvh[4 * ref];
                nb = sc.bvh[4 * ref + 1];
                nc = sc.bvh[4 * ref + 2];
                nr = reinterpret_cast<const uint4*>(sc.bvh)[4 * ref + 3];
              }
              const Slab sl = slab3_fused(xyz(na), xyz(nb), oinv, invc);
              const Slab sr = slab3_fused(V3{na.w, nc.x, nc.y}, V3{nb.w, nc.z, nc.w}, oinv, invc);
              const bool hl = (sl.tn <= sl.tf) & (sl.tf >= 0.001f) & (sl.tn <= closest);
              const bool hr = (sr.tn <= sr.tf) & (sr.tf >= 0.001f) & (sr.tn <= closest);
              if (hl & hr) {
                const bool lfirst = sl.tn <= sr.tn;
                tstack[depth_s * kBlock + tid] = lfirst ? nr.y : nr.x;
                ++depth_s;
                ref = lfirst ? nr.x : nr.y;
              } else if (hl | hr) {
                ref = hl ? nr.x : nr.y;
              } else {
                ref = depth_s ? tstack[--depth_s * kBlock + tid] : kBvhEnd;
              }
            }
            if (ref == kBvhEnd) break;
            DIAG_WAVE(DG_LEAF_W);
            DIAG_LANE(DG_LEAF_L);
            // leaf: slots [first, first + count) of the leaf-order records
            const uint32_t first = ref & ((1u << kBvhSlotBits) - 1u);
            const uint32_t cnt = ((ref >> kBvhSlotBits) & 15u) + 1u;
            for (uint32_t kk = 0; kk < cnt; ++kk) {
              const uint32_t slot = first + kk;
              const uint32_t i = sc.bvh_order[slot];
              const float4* r = sc.lrec + 4 * slot;
              const float tmax =
                  static_cast<int>(i) < best ? __uint_as_float(__float_as_uint(closest) + 1u) : closest;
              const uint32_t k = KS == KS_AABB ? FR_AABB : KS == KS_SPHERE ? FR_SPHERE : __float_as_uint(r[3].w);
              float t = 0.0f;
              bool h = false;
              if (k == FR_SPHERE) {
                const float4 g = r[0];
#ifndef FR_SPHERE_IEEE
                h = sphere_root_fast(xyz(g), g.w, o, d, a_dd, ssg, 0.001f, tmax, t);
#else
                h = sphere_root(xyz(g), g.w, o, d, a_dd, 0.001f, tmax, t);
#endif
              } else if (k == FR_AABB) {
                h = slab_root(slab3(xyz(r[0]), xyz(r[1]), o, inv), 0.001f, tmax, t);
              } else if (k == FR_TRIANGLE) {
                h = tri_root(xyz(r[0]), xyz(r[1]), xyz(r[2]), o, d, 0.001f, tmax, t);
              } else if (k == FR_OBB) {
                const float4 a = r[0], b = r[1], c = r[2], e = r[3];
                const ObbFrame f = obb_frame(xyz(a), xyz(b), xyz(c), xyz(e), o, d);
                h = slab_root(slab3(V3{-a.w, -b.w, -c.w}, V3{a.w, b.w, c.w}, f.ol, f.inv), 0.001f, tmax, t);
              }
              if (h) {
                closest = t;
                best = static_cast<int>(i);
                if (HAS_PLANE) t_last = t;
              }
            }
            ref = depth_s ? tstack[--depth_s * kBlock + tid] : kBvhEnd;
          }
        }
      }
      // one primitive of kind K at list index i (wave-uniform): records by scalar loads
      auto test_one = [&](auto kind_tag, uint32_t i) {
        constexpr uint32_t K = decltype(kind_tag)::value;
        const RecRef r4 = rec_at(sc.rec, i);  // scalar loads
        float t = 0.0f;
        bool h = false;
        if constexpr (K == FR_AABB) {
          h = slab_root(slab3(xyz(r4[0]), xyz(r4[1]), o, inv), 0.001f, closest, t);
        } else if constexpr (K == FR_SPHERE) {
          const float4 g = r4[0];
#ifndef FR_SPHERE_IEEE
          h = sphere_root_fast(xyz(g), g.w, o, d, a_dd, ssg, 0.001f, closest, t);
#else
          h = sphere_root(xyz(g), g.w, o, d, a_dd, 0.001f, closest, t);
#endif
        } else if constexpr (K == FR_PLANE) {
          const int r = plane_test(xyz(r4[0]), xyz(r4[1]), xyz(r4[2]), o, d, 0.001f, closest, t);
          if (r) t_last = t;
          h = r == 2;
        } else if constexpr (K == FR_TRIANGLE) {
          h = tri_root(xyz(r4[0]), xyz(r4[1]), xyz(r4[2]), o, d, 0.001f, closest, t);
        } else if constexpr (K == FR_OBB) {
          const float4 a = r4[0], b = r4[1], c = r4[2], e = r4[3];
          const ObbFrame f = obb_frame(xyz(a), xyz(b), xyz(c), xyz(e), o, d);
          h = slab_root(slab3(V3{-a.w, -b.w, -c.w}, V3{a.w, b.w, c.w}, f.ol, f.inv), 0.001f, closest, t);
        }
        if (h) {
          closest = t;
          best = static_cast<int>(i);
          if (HAS_PLANE) t_last = t;
        }
      };
      typedef std::integral_constant<uint32_t, FR_AABB> TagAabb;
      typedef std::integral_constant<uint32_t, FR_SPHERE> TagSphere;
#ifndef FR_NO_UNROLL_NIB
      if constexpr (NIB && KS != KS_ANY) {
        // <= kNibbleMaxPrims primitives: the tests unrolled over the compile-time bound with
        // an exit at n, each index an inline constant (the winner select needs no index
        // register) and each record at a constant offset. C3 trace 17.45 -> 17.29 ms as a
        // counted loop with an exit, -> 16.95 ms unrolled; shard 0/8 -1.6 %
        auto test_k = [&](auto ic) {
          if constexpr (KS == KS_AABB)
            test_one(TagAabb{}, decltype(ic)::value);
          else
            test_one(TagSphere{}, decltype(ic)::value);
        };
        // n through an empty asm here: otherwise the 15 tests' exit conditions are hoisted
        // out of the lane loop as lane masks held (and spilled) in SGPRs
        uint32_t n_here = sc.n;
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" : "+s"(n_here));
#endif
        unroll_below<0u, kNibbleMaxPrims>(n_here, test_k);
      } else
#endif
      if constexpr (KS != KS_ANY) {
        for (uint32_t ii = 0; ii < (list_walk ? sc.n : 0u); ++ii) {
          // the index is wave-uniform; say so, or the compiler may fall back to vector loads
          const uint32_t i = __builtin_amdgcn_readfirstlane(ii);
          if constexpr (KS == KS_AABB)
            test_one(TagAabb{}, i);
          else
            test_one(TagSphere{}, i);
        }
      } else {
        // The list in order, as its kind runs: one scalar kind branch per run instead of a
        // dependent kind load and branch per primitive, and a tight loop per run whose
        // record loads do not wait on a kind test (the same tests in the same order).
        typedef __attribute__((address_space(4))) const uint32_t cu32r;
        for (uint32_t rr = 0; rr < (list_walk ? sc.n_runs : 0u); ++rr) {
          const cu32r* rp = (cu32r*)(reinterpret_cast<uintptr_t>(sc.runs)) + 4u * __builtin_amdgcn_readfirstlane(rr);
          const uint32_t k = rp[0], i0 = rp[1], i1 = rp[2];
          if (k == FR_AABB) {
            for (uint32_t i = i0; i < i1; ++i) test_one(TagAabb{}, __builtin_amdgcn_readfirstlane(i));
          } else if (k == FR_SPHERE) {
            for (uint32_t i = i0; i < i1; ++i) test_one(TagSphere{}, __builtin_amdgcn_readfirstlane(i));
          } else if (k == FR_PLANE) {
            for (uint32_t i = i0; i < i1; ++i)
              test_one(std::integral_constant<uint32_t, FR_PLANE>{}, __builtin_amdgcn_readfirstlane(i));
          } else if (k == FR_TRIANGLE) {
            for (uint32_t i = i0; i < i1; ++i)
              test_one(std::integral_constant<uint32_t, FR_TRIANGLE>{}, __builtin_amdgcn_readfirstlane(i));
          } else if (k == FR_OBB) {
            for (uint32_t i = i0; i < i1; ++i)
              test_one(std::integral_constant<uint32_t, FR_OBB>{}, __builtin_amdgcn_readfirstlane(i));
          }  // FR_STUB: never hits (aabb.rs:21-34, rectangle.rs:21-34)
        }
      }
      PROF_MARK(PF_HIT);
      if (best < 0) {
        if (DEFER)
#ifdef FR_FAST_SKY
          tsky = __float_as_uint(sky_t_fast(d));  // tracer.rs:211-218, the blend in sum_kernel
#else
          tsky = __float_as_uint(sky_t(d));  // tracer.rs:211-218, the blend in sum_kernel
#endif
        else
          term = sky(d);  // tracer.rs:211-218
        ended = true;
        have_ray = false;
      } else {
        DIAG_WAVE(DG_HIT_W);
        ++nhit;
        ended = true;  // unless a scatter continues the path
        have_ray = false;
        if (depth < kp.max_depth) {
          // the shared HitRecord: normal of the winner at its own t; p = point_at(last t written)
          const V3 pw = add(o, scl(closest, d));
          // the winner's record and class: LDS when staged (n_rec / n_att are uniform;
          // separate branches keep LDS and global reads in their own address spaces)
          float4 b0, b1, b2, b3;
          if (REC_LDS || n_rec) {
            const float4* rb = rec_lds + 4 * best;
            b0 = rb[0];
            b1 = rb[1];
            b2 = rb[2];
            b3 = rb[3];
          } else {
            const uint32_t off = 64u * static_cast<uint32_t>(best);
            b0 = buf_load4(sc.rec, off);
            b1 = buf_load4(sc.rec, off + 16u);
            b2 = buf_load4(sc.rec, off + 32u);
            b3 = buf_load4(sc.rec, off + 48u);
          }
          // (a single-kind scene has no stubs: with DIFFUSE every class scatters lambertian)
          const uint32_t c = (DIFFUSE && KS != KS_ANY) ? static_cast<uint32_t>(SC_LAMBERT)
                             : ATT_LDS || n_att        ? __float_as_uint(att_lds[best].w)
                                                       : buf_load1(sc.cls, 4u * best);
          const uint32_t kb = KS == KS_AABB ? FR_AABB : KS == KS_SPHERE ? FR_SPHERE : __float_as_uint(b3.w);
          V3 n;
          if (kb == FR_AABB) {
            n = slab_normal(slab3(xyz(b0), xyz(b1), o, inv), closest, d);
          } else if (kb == FR_SPHERE) {
            n = divs(sub(pw, xyz(b0)), b0.w);
          } else if (kb == FR_PLANE) {
            n = scl(-1.0f, xyz(b1));
          } else if (kb == FR_TRIANGLE) {
            // precomputed winding normal, turned to face the ray except for dielectric
            n = xyz(b3);
            if (c != SC_DIELECTRIC && dot(n, d) > 0.0f) n = scl(-1.0f, n);
          } else {
            const ObbFrame f = obb_frame(xyz(b0), xyz(b1), xyz(b2), xyz(b3), o, d);
            const Slab sl = slab3(V3{-b0.w, -b1.w, -b2.w}, V3{b0.w, b1.w, b2.w}, f.ol, f.inv);
            n = obb_normal(xyz(b1), xyz(b2), xyz(b3), sl, closest, f.dl);
          }
          const V3 p = HAS_PLANE ? add(o, scl(t_last, d)) : pw;
          // Written for every hit lane, so that only the rarer materials' values are set
          // under a branch (fewer register copies where the branches join): an absorbed
          // path (SC_NONE) ends here and its o, d and sbest are not read again.
          const V3 din = d;
          o = p;
          d = add(p, n);  // lambertian / light: target = (p + n) + rus
          sbest = static_cast<uint32_t>(best);
          smetal = !DIFFUSE && c == SC_METAL;
          ended = c == SC_NONE;
          if (c != SC_NONE && (DIFFUSE || c != SC_DIELECTRIC)) need = NEED_SPHERE;
          if (!DIFFUSE && c == SC_DIELECTRIC) {
            // one draw, no rejection loop (sphere.rs:107-145)
            d = scatter_dielectric(din, n, rng);
            push(static_cast<uint32_t>(best));
            ++depth;
            ++nscat;
            have_ray = true;
          } else if (smetal) {
            // metal: reflect(unit(d), n) + fuzz * rus
            sfuzz = sc.mat[best].w;
            sn = n;
            d = reflect(unit(din), n);
          }
        }
      }
    }
    PROF_MARK(PF_SHADE);
    if (ended) {
      // 3. attenuation * get_color(...) (tracer.rs:206-207), innermost first
      DIAG_WAVE(DG_END_W);
      DIAG_LANE(DG_END_L);
      V3 col = term;
      if (NIB) {
        col = V3{__uint_as_float(tsky), __uint_as_float(wnib), 0.0f};
        wnib = ~0u;  // the next sample starts empty
      } else if (DEFER) {
        const uint2 w = *drow;
        *drow = make_uint2(~0u, ~0u);  // the next sample starts empty
        col = V3{__uint_as_float(tsky), __uint_as_float(w.x), __uint_as_float(w.y)};
      } else if (MAXD > 0) {
        // One read brings the lane's 8 levels; empty ones point at the unit entry
        // (x * 1.0f == x), so the product a0*(a1*(...*term)) needs no per-level branch
        // and its reads do not wait on each other.
        const uint4 w = *hrow;
        *hrow = make_uint4(unit2, unit2, unit2, unit2);  // the next sample starts empty
        const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
        if (n_att) {
          const char* att_bytes = reinterpret_cast<const char*>(att_lds);
#pragma unroll
          for (int j = MAXD - 1; j >= 0; --j) {
            DIAG_WAVE(DG_UNW_W);
            const uint32_t off = (j & 1) ? (ws[j >> 1] >> 16) : (ws[j >> 1] & 0xFFFFu);  // byte offset
            col = mul(xyz(*reinterpret_cast<const float4*>(att_bytes + off)), col);
          }
        } else {
          // global attenuations: only the levels in use
#pragma unroll
          for (int j = MAXD - 1; j >= 0; --j)
            if (j < static_cast<int>(depth)) col = mul(xyz(sc.att[(ws[j >> 1] >> (16 * (j & 1))) & 0xFFFFu]), col);
        }
      } else {
        // An absorbed path (terminal colour +0) stays +0 through any chain of finite,
        // non-negative attenuations: skip its unwind (sc.att_nonneg is the host's check).
        const bool zero_term = (__float_as_uint(term.x) | __float_as_uint(term.y) | __float_as_uint(term.z)) == 0u;
        const int udepth = sc.att_nonneg && zero_term ? 0 : static_cast<int>(depth);
        if (n_att) {
          for (int j = udepth - 1; j >= 0; --j) {
            const uint32_t pi = stack[j * kBlock + tid];
            col = mul(xyz(att_lds[pi]), col);
          }
        } else {
          for (int j = udepth - 1; j >= 0; --j) col = mul(xyz(sc.att[stack[j * kBlock + tid]]), col);
        }
      }
      if (!staged) {
        out[WPS * jj] = col.x;
        out[WPS * jj + 1] = col.y;
        if (WPS == 3) out[WPS * jj + 2] = col.z;
      } else {
        // stage the colour; every STG-th sample of the block, and its last, go out together
        float* sl = stage + WPS * (jj & (STG - 1u));
        sl[0] = col.x;
        sl[1] = col.y;
        if (WPS == 3) sl[2] = col.z;
        const bool full = (jj & (STG - 1u)) == STG - 1u;
        if (full || s + 1u == s_end) {
          float* dst = out + WPS * (jj & ~(STG - 1u));
          if (full && kp.ks == kBlockSamples) {
            if constexpr ((WPS * STG) % 4u == 0u) {
              // 16-B aligned: item * 192 (128) B + a multiple of 48 (32) B
              const float4* src = reinterpret_cast<const float4*>(stage);
#pragma unroll
              for (uint32_t k = 0; k < WPS * STG / 4u; ++k) reinterpret_cast<float4*>(dst)[k] = src[k];
            } else {
              // 8-B aligned: item * 192 B + a multiple of 24 B
              const float2* src = reinterpret_cast<const float2*>(stage);
#pragma unroll
              for (uint32_t k = 0; k < WPS * STG / 2u; ++k) reinterpret_cast<float2*>(dst)[k] = src[k];
            }
          } else {
            for (uint32_t k = 0; k < WPS * ((jj & (STG - 1u)) + 1u); ++k) dst[k] = stage[k];
          }
        }
      }
      ++jj;
#ifdef FR_DIAG
      if (s + 1u == s_end && diag_tb < (1u << 20)) atomicAdd(&g_fr_tb_cost[diag_tb], nseg - diag_seg0);
#endif
      if (++s == s_end)
        need_item = true;
      else
        need_jit = true;  // next sample of the block, same stream
    }
    PROF_MARK(PF_END);
  }

  // Per-wave counter reduction into the wave's own slot (plain stores): the waves leave
  // the drain within a fraction of a millisecond, and three returning atomics per wave on
  // one cache line queued long enough there to hold the kernel's end back.
  unsigned long long a = nseg, b = nhit, sct = nscat;
  for (int m = 32; m > 0; m >>= 1) {
    a += __shfl_xor(a, m);
    b += __shfl_xor(b, m);
    sct += __shfl_xor(sct, m);
  }
  if (lane == 0) {
    unsigned long long* wc = kw.wave_counters + 3u * (blockIdx.x * (kBlock / 64u) + (tid >> 6));
    wc[0] = a;
    wc[1] = b;
    wc[2] = sct;
  }
#ifdef FR_PROF
  if (lane == 0)
    for (int k = 0; k < PF_N; ++k) atomicAdd(&kw.counters[20 + k], static_cast<unsigned long long>(pf_acc[k]));
#endif
#ifdef FR_DIAG
  if (lane == 0 && gw < 65536) {
    g_fr_wave_times[2 * gw + 1] = __builtin_amdgcn_s_memrealtime();
    g_fr_wave_iters[2 * gw + 1] = diag_iter;
  }
  __syncthreads();
  if (tid < DG_N) atomicAdd(&kw.counters[4 + tid], static_cast<unsigned long long>(dg[tid]));
#endif
}

// Adds each pixel's sample colours of this pass, in sample order, onto its running
// sum (tracer.rs:174); the last pass divides by spp, gamma-corrects and quantises
// (tracer.rs:177-184). One thread per pixel slot. A workgroup's 256 slots of one sample
// block are one contiguous run of the item-major buffer (256 x 192 B, or 128 B for 8-B
// records, at ks = 16): it is
// read with coalesced 16-B loads into an LDS tile whose odd slot stride keeps each
// thread's reads of its own slot bank-conflict free, then summed in sample order. With
// KF_DEFER the slots hold deferred-unwind records (kDeferUnit) and the colour is rebuilt
// here from a 12-B-per-entry attenuation table (tile + table fit three workgroups per CU).
// WPS = 2: 8-B records {t, 4-bit winners} (KF_NIBBLE).
constexpr uint32_t kSumThreads = 256;

template <uint32_t WPS>
__global__ __launch_bounds__(kSumThreads) void sum_kernel(KParams kp, const float* __restrict__ samples,
                                                          float* __restrict__ running, float* __restrict__ out_mean,
                                                          uint8_t* __restrict__ out_u8, int first, int last,
                                                          const float4* __restrict__ att, uint32_t n_prims) {
  constexpr uint32_t kSumSlot = WPS * kBlockSamples + 1;  // floats per slot in LDS (odd stride)
  __shared__ float tile[kSumThreads * kSumSlot];
  __shared__ float att_s[3 * (kDeferUnit + 1)];  // KF_DEFER: attenuation rgb, entry kDeferUnit = 1
  const uint32_t t = threadIdx.x;
  const bool defer = (kp.flags & KF_DEFER) != 0;
  if (defer) {  // kSumThreads == kDeferUnit + 1
    const float4 a = t < n_prims ? att[t] : make_float4(1.0f, 1.0f, 1.0f, 0.0f);
    att_s[3 * t] = a.x;
    att_s[3 * t + 1] = a.y;
    att_s[3 * t + 2] = a.z;
  }
  const uint32_t q0 = blockIdx.x * kSumThreads, q = q0 + t;
  const uint32_t nq = min(kSumThreads, kp.P - q0);
  uint32_t x = 0, y = 0;
  const bool valid = q < kp.P && slot_xy(kp, q, x, y);
  const bool mt = (kp.flags & FR_FLAG_MT_BANDS) != 0;
  const bool mt_zero = mt && !(kp.band_h && y / kp.band_h < 4u);  // rows render_mt never fills stay 0
  V3 sum = (first || !valid) ? V3{0.0f, 0.0f, 0.0f} : V3{running[3 * q], running[3 * q + 1], running[3 * q + 2]};
  const float fspp = static_cast<float>(kp.spp);
  const uint32_t per = WPS * kp.ks;  // floats per slot in the buffer
  // full 16-sample slots: block bl + 1's loads are issued before block bl is summed, so
  // they are in flight during the sum (a shard at N = 8 gives each workgroup's thread a
  // chain of 16 dependent block loads)
  constexpr uint32_t kV = WPS * kBlockSamples / 4u;  // float4 per slot
  const uint32_t n4 = nq * kV;
  float4 v[kV];
  auto load_block = [&](uint32_t bl) {
    // 192-B (128-B) slots: 16-B aligned
    const float4* src4 = reinterpret_cast<const float4*>(samples + WPS * (static_cast<size_t>(bl * kp.P + q0) * kp.ks));
#pragma unroll
    for (uint32_t k = 0; k < kV; ++k) {
      const uint32_t i = t + k * kSumThreads;
      if (i < n4) v[k] = src4[i];
    }
  };
  if (kp.ks == kBlockSamples && kp.nb) load_block(0);
  for (uint32_t bl = 0; bl < kp.nb; ++bl) {
    const float* src = samples + WPS * (static_cast<size_t>(bl * kp.P + q0) * kp.ks);
    __syncthreads();  // the previous block's reads are done (and the table is written)
    if (kp.ks == kBlockSamples) {
#pragma unroll
      for (uint32_t k = 0; k < kV; ++k) {
        const uint32_t i = t + k * kSumThreads;
        if (i < n4) {
          const uint32_t slot = i / kV, w = (i - slot * kV) * 4u;
          float* d = tile + slot * kSumSlot + w;
          d[0] = v[k].x;
          d[1] = v[k].y;
          d[2] = v[k].z;
          d[3] = v[k].w;
        }
      }
      if (bl + 1u < kp.nb) load_block(bl + 1u);
    } else {
      for (uint32_t i = t; i < nq * per; i += kSumThreads) tile[(i / per) * kSumSlot + i % per] = src[i];
    }
    __syncthreads();
    if (valid && !mt_zero) {
      const uint32_t n = min(kBlockSamples, kp.spp - (kp.b0 + bl) * kBlockSamples);
      const float* c = tile + t * kSumSlot;
      for (uint32_t j = 0; j < n; ++j, c += WPS) {
        if (WPS == 2) {
          // 8-B record: terminal, then a_7 ... a_0 from 4-bit entries (kNibbleUnit: 1)
          const uint32_t tb = __float_as_uint(c[0]), w = __float_as_uint(c[1]);
          V3 col = tb == kDeferAbsorbed ? V3{0.0f, 0.0f, 0.0f} : sky_from_t(c[0]);
#pragma unroll
          for (int k = 7; k >= 0; --k) {
            const float* e = att_s + 3u * ((w >> (4 * k)) & 0xFu);
            col = mul(V3{e[0], e[1], e[2]}, col);
          }
          sum = add(sum, col);
        } else if (defer) {
          // the deferred unwind (kDeferUnit): terminal, then a_7 ... a_0 innermost first
          const uint32_t tb = __float_as_uint(c[0]), lo = __float_as_uint(c[1]), hi = __float_as_uint(c[2]);
          V3 col = tb == kDeferAbsorbed ? V3{0.0f, 0.0f, 0.0f} : sky_from_t(c[0]);
#pragma unroll
          for (int k = 7; k >= 0; --k) {
            const float* e = att_s + 3u * (((k >= 4 ? hi : lo) >> (8 * (k & 3))) & 0xFFu);
            col = mul(V3{e[0], e[1], e[2]}, col);
          }
          sum = add(sum, col);
        } else if (mt) {  // save_image_mt (tracer.rs:140-145): acc += (sqrt(c) * 255) as u8 / sample
          sum = add(sum, V3{static_cast<float>(to_u8(c[0])) / fspp, static_cast<float>(to_u8(c[1])) / fspp,
                            static_cast<float>(to_u8(c[2])) / fspp});
        } else {
          sum = add(sum, V3{c[0], c[1], c[2]});
        }
      }
    }
  }
  if (!valid) return;
  if (mt_zero) {
    if (last) {
      const size_t idx = (static_cast<size_t>(y) * kp.W + x) * 3u;
      for (int ch = 0; ch < 3; ++ch) {
        out_mean[idx + ch] = 0.0f;
        out_u8[idx + ch] = 0;
      }
    }
    return;
  }
  if (!last) {
    running[3 * q] = sum.x;
    running[3 * q + 1] = sum.y;
    running[3 * q + 2] = sum.z;
    return;
  }
  const size_t idx = (static_cast<size_t>(y) * kp.W + x) * 3u;
  if (mt) {  // tracer.rs:148-155: `pixels_acc as u8`
    out_mean[idx + 0] = sum.x;
    out_mean[idx + 1] = sum.y;
    out_mean[idx + 2] = sum.z;
    out_u8[idx + 0] = as_u8_trunc(sum.x);
    out_u8[idx + 1] = as_u8_trunc(sum.y);
    out_u8[idx + 2] = as_u8_trunc(sum.z);
    return;
  }
  const V3 mean = divs(sum, static_cast<float>(kp.spp));  // tracer.rs:177
  out_mean[idx + 0] = mean.x;
  out_mean[idx + 1] = mean.y;
  out_mean[idx + 2] = mean.z;
  if (kp.flags & FR_FLAG_WRITE_U8) {
    out_u8[idx + 0] = to_u8(mean.x);
    out_u8[idx + 1] = to_u8(mean.y);
    out_u8[idx + 2] = to_u8(mean.z);
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
    case 12: r = fmin_num(fmin_num(x, y), b[(i + 1) % n]); break;
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
  std::vector<unsigned char> host(off, 0);
  bool nonneg = true;
  bool diffuse = true;
  if (!bvh_nodes.empty()) memcpy(&host[c->off_bvh], bvh_nodes.data(), bvh_nodes.size() * sizeof(BvhNode));
  if (!bvh_order.empty()) memcpy(&host[c->off_bvh_order], bvh_order.data(), bvh_order.size() * 4);
  if (!bvh_segs.empty()) memcpy(&host[c->off_segs], bvh_segs.data(), bvh_segs.size() * sizeof(BvhSegment));
  if (!runs.empty()) memcpy(&host[c->off_runs], runs.data(), runs.size() * 4);
  c->bvh_ok = bvh_ok;
  c->bvh_extent = bvh_extent;
  c->n_segs = static_cast<uint32_t>(bvh_segs.size());
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
    for (float a : {att.x, att.y, att.z})
      if (!(a >= 0.0f) || std::signbit(a) || !std::isfinite(a)) nonneg = false;
    memcpy(&g[3].w, &kind, 4);  // kind bits in g3.w
    memcpy(&host[c->off_rec + 64 * i], g, 64);
  }
  c->att_nonneg = nonneg;
  c->diffuse = diffuse;
  // the BVH leaves' records, in leaf-slot order
  for (size_t slot = 0; slot < bvh_order.size(); ++slot)
    memcpy(&host[c->off_lrec + 64 * slot], &host[c->off_rec + 64 * static_cast<size_t>(bvh_order[slot])], 64);
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
  unsigned long long* d_cnt = nullptr;  // [0..3] counters, [4..] diagnostics; [31] queue head
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
  std::chrono::steady_clock::time_point t0;
  // fr_ctx_trace_log: event pairs around every trace launch since the log was enabled,
  // across renders (ev_trace holds only the last render's), so a caller streaming K
  // frames can average the kernel's duration over all of them
  // log 0: trace launches (on the launch's stream); log 1: whole renders (ev0 .. ev1)
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
};

template <typename Kern>
static void launch_persistent(Kern kern, const Grid& g, size_t lds, hipStream_t st, KArgs a) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, static_cast<int>(kBlock), lds) != hipSuccess ||
      per_cu < 1)
    per_cu = 1;
  // the per-wave counter slots (fr_ctx::d_wcnt) hold kMaxWgPerCu workgroups per CU
  if (per_cu > static_cast<int>(kMaxWgPerCu)) per_cu = static_cast<int>(kMaxWgPerCu);
  // FR_BVH_STAGE: "0" BVH kernels store unstaged, "1" staged even at a lower residency (A/B, tests)
  const char* stage_env = getenv("FR_BVH_STAGE");
  const bool force_stage = stage_env && strcmp(stage_env, "1") == 0;
  if (g.stage_bytes && !(stage_env && strcmp(stage_env, "0") == 0)) {
    int staged = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&staged, kern, static_cast<int>(kBlock), lds + g.stage_bytes) ==
            hipSuccess &&
        (staged >= per_cu || (force_stage && staged >= 1))) {
      per_cu = staged < static_cast<int>(kMaxWgPerCu) ? staged : static_cast<int>(kMaxWgPerCu);
      lds += g.stage_bytes;
      a.kp.flags |= KF_STAGE;
    }
  }
  *g.per_cu = per_cu;
  uint64_t cap = static_cast<uint64_t>(per_cu) * static_cast<uint64_t>(g.num_cus);
  // FR_MAX_WGS=k caps the grid (tests: with a few workgroups every wave claims many
  // batches, partly used ones included, so the claim paths run at small image sizes)
  if (const char* e = getenv("FR_MAX_WGS"))
    if (atoi(e) > 0 && static_cast<uint64_t>(atoi(e)) < cap) cap = static_cast<uint64_t>(atoi(e));
  const uint32_t blocks = static_cast<uint32_t>(g.want < cap ? (g.want ? g.want : 1u) : cap);
  *g.blocks = blocks;
  a.kp.n_static = blocks * kBlock;  // one 64-item batch per wave of the grid
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(kBlock), lds, st, a);
}

template <int KS, bool HP, bool BV, bool MT = false>
static void launch_depth(bool small_depth, const Grid& g, size_t lds, hipStream_t st, const KScene& ks,
                         const KCam& kc, const KParams& kp, const KWork& kw) {
  if constexpr (!BV && !MT) {
    if (kp.flags & KF_DEFER) {
      if ((kp.flags & KF_NIBBLE) && (kp.flags & KF_DIFFUSE))
        launch_persistent(trace_kernel<KS, HP, FR_KREJ_NIB, kSmallDepth, false, false, 2, 1>, g, lds, st,
                          KArgs{ks, kc, kp, kw});
      else if (kp.flags & KF_NIBBLE)
        launch_persistent(trace_kernel<KS, HP, FR_KREJ_NIB, kSmallDepth, false, false, 2>, g, lds, st,
                          KArgs{ks, kc, kp, kw});
      else if (kp.flags & KF_DIFFUSE)
        launch_persistent(trace_kernel<KS, HP, FR_KREJ, kSmallDepth, false, false, 1, 1>, g, lds, st,
                          KArgs{ks, kc, kp, kw});
      else
        launch_persistent(trace_kernel<KS, HP, FR_KREJ, kSmallDepth, false, false, 1>, g, lds, st,
                          KArgs{ks, kc, kp, kw});
      return;
    }
  }
  const bool diffuse = (kp.flags & KF_DIFFUSE) != 0;
  if (small_depth && diffuse)
    launch_persistent(trace_kernel<KS, HP, FR_KREJ, kSmallDepth, BV, MT, 0, 1>, g, lds, st, KArgs{ks, kc, kp, kw});
  else if (small_depth)
    launch_persistent(trace_kernel<KS, HP, FR_KREJ, kSmallDepth, BV, MT, 0>, g, lds, st, KArgs{ks, kc, kp, kw});
  else if (diffuse)
    launch_persistent(trace_kernel<KS, HP, FR_KREJ, 0, BV, MT, 0, 1>, g, lds, st, KArgs{ks, kc, kp, kw});
  else
    launch_persistent(trace_kernel<KS, HP, FR_KREJ, 0, BV, MT, 0>, g, lds, st, KArgs{ks, kc, kp, kw});
}

// BVH kernels walk the list's segments (bvh.h); scenes with planes use the general
// kernel, which tests each plane in list order between the runs.
static void launch_trace(uint32_t kinds, bool has_plane, bool bvh, bool small_depth, const Grid& g, size_t lds,
                         hipStream_t st, const KScene& ks, const KCam& kc, const KParams& kp, const KWork& kw) {
  if (kp.flags & FR_FLAG_MT_BANDS) {  // save_image_mt: the general kernels, in-order loop
    if (has_plane)
      launch_depth<KS_ANY, true, false, true>(small_depth, g, lds, st, ks, kc, kp, kw);
    else
      launch_depth<KS_ANY, false, false, true>(small_depth, g, lds, st, ks, kc, kp, kw);
  } else if (kinds == (1u << FR_AABB)) {
    if (bvh)
      launch_depth<KS_AABB, false, true>(small_depth, g, lds, st, ks, kc, kp, kw);
    else
      launch_depth<KS_AABB, false, false>(small_depth, g, lds, st, ks, kc, kp, kw);
  } else if (kinds == (1u << FR_SPHERE)) {
    if (bvh)
      launch_depth<KS_SPHERE, false, true>(small_depth, g, lds, st, ks, kc, kp, kw);
    else
      launch_depth<KS_SPHERE, false, false>(small_depth, g, lds, st, ks, kc, kp, kw);
  } else if (has_plane) {
    if (bvh)
      launch_depth<KS_ANY, true, true>(small_depth, g, lds, st, ks, kc, kp, kw);
    else
      launch_depth<KS_ANY, true, false>(small_depth, g, lds, st, ks, kc, kp, kw);
  } else if (bvh) {
    launch_depth<KS_ANY, false, true>(small_depth, g, lds, st, ks, kc, kp, kw);
  } else {
    launch_depth<KS_ANY, false, false>(small_depth, g, lds, st, ks, kc, kp, kw);
  }
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
      hipMalloc(&c->d_cnt, 32 * sizeof(unsigned long long)) != hipSuccess ||
      hipMalloc(&c->d_wcnt, 2 * 3 * sizeof(unsigned long long) * kMaxWgPerCu * (kBlock / 64u) * c->num_cus) !=
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

int fr_ctx_render(fr_ctx* c, fr_scene* scene, const fr_camera* cam, const fr_params* p) {
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
  KCam kc{cam->position[0], cam->position[1], cam->position[2], cam->lower_left[0], cam->lower_left[1],
          cam->lower_left[2], cam->horizontal[0], cam->horizontal[1], cam->horizontal[2], cam->vertical[0],
          cam->vertical[1], cam->vertical[2], cam->u[0], cam->u[1], cam->u[2], cam->v[0], cam->v[1], cam->v[2],
          cam->lens_radius};
  KParams kp;
  kp.W = p->width;
  kp.H = p->height;
  kp.rW = 1.0f / static_cast<float>(p->width);
  kp.rH = 1.0f / static_cast<float>(p->height);
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
  // §4.5a), so one pass is the default.
  // sample slots per item: a frame of spp < 16 (update()'s 1-spp frames) needs only spp
  kp.ks = p->spp < kBlockSamples ? (p->spp ? p->spp : 1u) : kBlockSamples;
  const bool small_depth = p->max_depth <= kSmallDepth && dc->n < 65536u;
  // the deferred unwind (kDeferMaxPrims); FR_DEFER=0 keeps the unwind in the trace kernel,
  // FR_DEFER=1 the 12-B records for small scenes too (A/B)
  const char* defer_env = getenv("FR_DEFER");
  const bool defer = small_depth && dc->n <= kDeferMaxPrims && !use_bvh && !(p->flags & FR_FLAG_MT_BANDS) &&
                     !(defer_env && strcmp(defer_env, "0") == 0);
  const bool nibble = defer && dc->n <= kNibbleMaxPrims && !(defer_env && strcmp(defer_env, "1") == 0);
  if (defer) kp.flags |= KF_DEFER;
  if (nibble) kp.flags |= KF_NIBBLE;
  // FR_MAT=0 keeps the general shading step for diffuse-only scenes (A/B, tests)
  const char* mat_env = getenv("FR_MAT");
  if (dc->diffuse && !(mat_env && strcmp(mat_env, "0") == 0)) kp.flags |= KF_DIFFUSE;
  const uint32_t wps = nibble ? 2u : 3u;  // words per sample in the buffer
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
  const int slots = passes > 1 ? 2 : 1;
  const size_t slot_bytes = per_block * nb_pass;
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
  const size_t stage_n = stage_samples(use_bvh);
  const size_t lds = (stage_n > 1 && !use_bvh ? kBlock * stage_n * wps * sizeof(float) : 0u) + (n_att ? n_att + 1 : 0) * 16 +
                     n_rec * 64 + stack_bytes + (use_bvh ? kBvhStack * kBlock * sizeof(uint32_t) : 0u);
  KWork kw;
  kw.counters = c->d_cnt;
  c->t0 = std::chrono::steady_clock::now();
  HIPCHK(hipMemsetAsync(c->d_cnt, 0, 32 * sizeof(unsigned long long), c->stream));
#ifdef FR_DIAG
  {
    const unsigned long long z[2] = {0, 0};
    HIPCHK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_fr_diag_lens), z, sizeof(z), 0, hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipMemcpyToSymbolAsync(HIP_SYMBOL(g_fr_diag_rus), z, sizeof(z), 0, hipMemcpyHostToDevice, c->stream));
    void* tc = nullptr;
    HIPCHK(hipGetSymbolAddress(&tc, HIP_SYMBOL(g_fr_tb_cost)));
    HIPCHK(hipMemsetAsync(tc, 0, (1u << 20) * sizeof(unsigned int), c->stream));
  }
#endif
  HIPCHK(hipEventRecord(c->ev0, c->stream));
  if (c->log_on) HIPCHK(log_start(c, 1, c->stream));
  HIPCHK(hipEventRecord(c->ev_start, c->stream));
  HIPCHK(hipStreamWaitEvent(c->stream2, c->ev_start, 0));
  HIPCHK(hipStreamWaitEvent(c->stream_sum, c->ev_start, 0));
  const uint32_t sum_blocks = (kp.P + kSumThreads - 1u) / kSumThreads;
  int traced = 0;  // trace launches whose events were recorded
  int summed = 0;
  for (int pass = 0; pass < passes || (pass == 0 && kp.P); ++pass) {
    const int slot = pass % 2;
    hipStream_t ts = slot ? c->stream2 : c->stream;
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
      kw.queue = reinterpret_cast<uint32_t*>(c->d_cnt + 31 - slot);
      kw.samples = samples;
      // persistent grid: the resident workgroup count (launch_persistent)
      uint32_t blocks = 0;
      const Grid grid{(static_cast<uint64_t>(kp.n_items) + kBlock - 1u) / kBlock, c->num_cus, &c->occupancy, &blocks,
                      use_bvh && stage_n > 1 ? kBlock * stage_n * 3 * sizeof(float) : 0u};
      unsigned long long* wcnt = c->d_wcnt + static_cast<size_t>(slot) * 3 * kMaxWgPerCu * (kBlock / 64u) * c->num_cus;
      kw.wave_counters = wcnt;
      HIPCHK(hipMemsetAsync(kw.queue, 0, sizeof(uint32_t), ts));
      HIPCHK(hipEventRecord(c->ev_trace[2 * traced], ts));
      if (c->log_on) HIPCHK(log_start(c, 0, ts));
      launch_trace(dc->kinds, dc->has_plane, use_bvh, small_depth, grid, lds, ts, ks, kc, kp, kw);
      HIPCHK(hipGetLastError());
      HIPCHK(hipEventRecord(c->ev_trace[2 * traced + 1], ts));
      if (c->log_on) HIPCHK(log_end(c, 0, ts));
      HIPCHK(hipStreamWaitEvent(c->stream_sum, c->ev_trace[2 * traced + 1], 0));
      // on the sum stream, after the trace: the frame's end (ev1 on c->stream) waits for
      // the sums, so fr_ctx_sync reads d_cnt after every pass's reduce, and the next
      // frame's d_cnt memset (c->stream) cannot overtake a reduce of this one
      hipLaunchKernelGGL(reduce_counters, dim3(1), dim3(256), 0, c->stream_sum, wcnt, blocks * (kBlock / 64u),
                         c->d_cnt);
      HIPCHK(hipGetLastError());
      ++traced;
    }
    const int first = pass == 0, last = pass + 1 >= passes;
    if (first && c->copy_pending) HIPCHK(hipStreamWaitEvent(c->stream_sum, c->ev_copy, 0));  // last gather done
    hipLaunchKernelGGL(nibble ? sum_kernel<2> : sum_kernel<3>, dim3(sum_blocks ? sum_blocks : 1u), dim3(kSumThreads), 0,
                       c->stream_sum, kp, samples,
                       c->d_running, c->d_mean, c->d_u8, first, last, ks.att, dc->n);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(c->ev_sum[pass], c->stream_sum));
    summed = pass + 1;
    if (last) break;
  }
  if (summed) HIPCHK(hipStreamWaitEvent(c->stream, c->ev_sum[summed - 1], 0));
  c->passes = traced;
  HIPCHK(hipEventRecord(c->ev1, c->stream));
  if (c->log_on) HIPCHK(log_end(c, 1, c->stream));
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
  if (st) {
    unsigned long long cnt[32] = {};
    HIPCHK(hipMemcpy(cnt, c->d_cnt, sizeof(cnt), hipMemcpyDeviceToHost));
#ifdef FR_PROF
    {
      double tot = 0;
      for (int k = 0; k < PF_N; ++k) tot += static_cast<double>(cnt[20 + k]);
      fprintf(stderr, "FR_PROF {\"claim\": %.4f, \"reject\": %.4f, \"hit\": %.4f, \"shade\": %.4f, \"end\": %.4f, "
              "\"wave_cycles\": %.4e}\n", cnt[20] / tot, cnt[21] / tot, cnt[22] / tot, cnt[23] / tot, cnt[24] / tot, tot);
    }
#endif
#ifdef FR_DIAG
    unsigned long long dl[2], dr[2];
    HIPCHK(hipMemcpyFromSymbol(dl, HIP_SYMBOL(g_fr_diag_lens), sizeof(dl)));
    HIPCHK(hipMemcpyFromSymbol(dr, HIP_SYMBOL(g_fr_diag_rus), sizeof(dr)));
    fprintf(stderr,
            "FR_DIAG {\"iter_w\": %llu, \"regen_w\": %llu, \"regen_l\": %llu, \"hit_w\": %llu, \"end_w\": %llu, "
            "\"end_l\": %llu, \"unwind_w\": %llu, \"unwind_l\": %llu, \"lens_w\": %llu, \"lens_l\": %llu, "
            "\"rus_w\": %llu, \"rus_l\": %llu, \"merged_w\": %llu, \"merged_l\": %llu, \"segments\": %llu, "
            "\"hits\": %llu, \"node_w\": %llu, \"node_l\": %llu, \"leaf_w\": %llu, \"leaf_l\": %llu}\n",
            cnt[4 + DG_ITER], cnt[4 + DG_REGEN_W], cnt[4 + DG_REGEN_L], cnt[4 + DG_HIT_W], cnt[4 + DG_END_W],
            cnt[4 + DG_END_L], cnt[4 + DG_UNW_W], cnt[4 + DG_UNW_L], dl[0], dl[1], dr[0], dr[1], cnt[4 + DG_LENS_W],
            cnt[4 + DG_LENS_L], cnt[0], cnt[1], cnt[4 + DG_NODE_W], cnt[4 + DG_NODE_L], cnt[4 + DG_LEAF_W],
            cnt[4 + DG_LEAF_L]);
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
    uint64_t rows = 0;
    for (uint32_t k = p.shard_index; k < strips; k += p.shard_count) {
      const uint32_t r0 = k * kStripRows, r1 = r0 + kStripRows < p.height ? r0 + kStripRows : p.height;
      rows += r1 - r0;
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
    st->scatters = cnt[2];
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

int fr_ctx_trace_log(fr_ctx* c, int enable) {
  if (!c) return set_error(FR_EARG, "fr_ctx_trace_log: null ctx");
  if (enable) {
    SET_DEVICE(c->device);
    // the pairs of an earlier log may still be pending on the streams: drain them before
    // their events are recorded again
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipStreamSynchronize(c->stream2));
    c->log_n[0] = c->log_n[1] = 0;
  }
  c->log_on = enable != 0;
  return FR_OK;
}

int fr_ctx_trace_log_read(fr_ctx* c, int which, double* ms, uint32_t cap, uint32_t* n) {
  if (!c || !n || which < 0 || which > 1) return set_error(FR_EARG, "fr_ctx_trace_log_read: bad argument");
  SET_DEVICE(c->device);
  HIPCHK(hipStreamSynchronize(c->stream));
  HIPCHK(hipStreamSynchronize(c->stream2));
  *n = static_cast<uint32_t>(c->log_n[which]);
  for (size_t i = 0; i < c->log_n[which] && i < cap && ms; ++i) {
    float t = 0.0f;
    HIPCHK(hipEventElapsedTime(&t, c->log_ev[which][2 * i], c->log_ev[which][2 * i + 1]));
    ms[i] = t;
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

}  // extern "C"
