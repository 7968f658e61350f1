// trace_kernel.h — the device side of the tracer: work-item mapping, kernel argument
// structs and the persistent path-tracing megakernel (trace_kernel).
//
// Compiled twice: into libforma_rt.so by hipcc (every specialisation, render.hip), and
// at run time by hiprtc for a scene-specialised list kernel (FR_JIT_N defined: the
// closest-hit list walk becomes an unrolled sequence of tests on the scene's records
// as compile-time constants, jit.cpp). Everything here must therefore
// compile under hiprtc: no host-only headers.
#pragma once
#if !defined(__HIPCC_RTC__)
#include <hip/hip_runtime.h>
#include <float.h>
#include <type_traits>
#include "../../include/forma_rt.h"
#include "bvh.h"
#else
#include <type_traits>
#include "forma_rt.h"
#include "bvh.h"
#ifndef FLT_MAX
#define FLT_MAX __FLT_MAX__
#endif
#endif

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

namespace fr {

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
// Re-tuned for the scene-specialised kernel (round 3): 9 with
// FR_CLAIM_MIN_NIB 3 streams C3 at 16.49 ms per frame against 16.63 (6 / 2), three runs;
// shard 0/8 unchanged (tools/gpu_knob_shards.sh, profiles/r03k_knob_shards.log)
#ifndef FR_KREJ_NIB
#define FR_KREJ_NIB 9
#endif
#ifndef FR_CLAIM_MIN
#define FR_CLAIM_MIN 1  // lanes that must wait for an item before the wave claims (tuning only)
#endif
// ... for the 8-B-record kernels (the headline's): C3 18.50 -> 18.28 ms at 2 (18.31 at 4, 18.46
// at 6); 4 on every kernel cost C2 +2 %, so the others keep FR_CLAIM_MIN
#ifndef FR_CLAIM_MIN_NIB
#define FR_CLAIM_MIN_NIB 3
#endif
// ... for the BVH kernels with 8-B attenuation-class records: C5 trace 39.51 -> 39.17 ms at 2
// (0: 39.87, 1: 39.27, 3: 39.31, 6: 40.14; profiles/r06af_ab_c5_krej.log, four runs)
#ifndef FR_KREJ_BVH
#define FR_KREJ_BVH 2
#endif
#ifndef FR_CLAIM_MIN_BVH
#define FR_CLAIM_MIN_BVH FR_CLAIM_MIN
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
// FR_SKY_DEFER builds (A/B): the 8-B-record kernel stores 12-B records {d.y, dot(d, d),
// winners} and sum_kernel computes the sky parameter, at full SIMD width, instead of the
// trace kernel in the few lanes whose path escapes in a given iteration. dot(d, d) = -1
// (which no sum of squares is) marks an absorbed path.
#ifdef FR_SKY_DEFER
constexpr bool kSkyDefer = true;
#else
constexpr bool kSkyDefer = false;
#endif
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

struct KScene {
  // one 64-B record per primitive (g0..g3; kind in the bits of g3.w): one scalar
  // load brings a primitive into SGPRs in the closest-hit loop
  const float4* __restrict__ rec;
  const float4* __restrict__ mat;   // colour rgb, fuzz
  const uint32_t* __restrict__ cls; // effective ScatterClass
  // attenuation class of each primitive (BVH kernels with 8-B records: the winners are
  // stored as classes, indices into a table of the scene's <= 15 distinct attenuations)
  const uint32_t* __restrict__ acls;
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
  // the jitter's (x + r) / W as 2^24 (x + r) / (2^24 W), the 2^24 folded into the operands
  // (exact scalings): rW = RN(1 / W) 2^-24 = RN(1 / (2^24 W)) (host IEEE division), sW =
  // 2^24 W; the same for H
  float rW, rH, sW, sH;
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
  float lens_s;       // lens 2^-23
  uint32_t lens_pre;  // lens_s is exact (no underflow): the lens sample uses it
};
static_assert(sizeof(KCam) == 21 * 4, "KCam is 21 words");

struct KArgs {
  KScene sc;
  KCam cam;
  KParams kp;
  KWork kw;
};

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
// (BVH kernels with 8-B records stage like the list kernels: their LDS holds no unwind stack)
__host__ __device__ constexpr uint32_t stage_samples(bool bvh, bool nib = false) {
  return bvh && !nib ? FR_BVH_STAGE : FR_STAGE;
}
// FR_BVH_SCALAR_NODES=1: a node step whose walking lanes are all at one node reads it with
// scalar loads (0, vector loads only: C5 trace 52.9 -> 62.3 ms, the vector memory path
// returning 64 B per lane per step)
#ifndef FR_STAGE_SMAJOR
#define FR_STAGE_SMAJOR 0  // slot-major sample staging for 8-B records (A/B knob)
#endif
#ifndef FR_BVH_SCALAR_NODES
#define FR_BVH_SCALAR_NODES 1
#endif
// FR_BVH_SCALAR_LEAVES=1: a leaf every lane is at is tested from scalar loads (A/B knob)
#ifndef FR_BVH_SCALAR_LEAVES
#define FR_BVH_SCALAR_LEAVES 1
#endif
// FR_BVH_RSTAGE=1: the BVH kernels hold a pair's first colour in registers instead of LDS
// (3 VGPRs, none of the traversal stack's LDS), so every BVH launch stores whole pairs.
#ifndef FR_BVH_RSTAGE
#define FR_BVH_RSTAGE 0
#endif
// A staging group larger than a sub-block (FR_STAGE 8): a sub-block's group store starts at
// the sub-block's first sample, so it never writes another sub-block's slots.
static_assert(kFineSamples % FR_STAGE == 0 || FR_STAGE % kFineSamples == 0, "staging groups and sub-blocks nest");
constexpr bool kStageSpansSub = FR_STAGE > kFineSamples;

// FR_DIAG builds count, per phase, wave-level trips (one per SIMT pass of the wave)
// and lane-level work, to measure SIMT efficiency. Never enabled in the product.
#ifdef FR_DIAG
enum { DG_ITER, DG_REGEN_W, DG_REGEN_L, DG_LENS_W, DG_LENS_L, DG_RUS_W, DG_RUS_L, DG_END_W, DG_END_L,
       DG_UNW_W, DG_UNW_L, DG_HIT_W, DG_NODE_W, DG_NODE_L, DG_LEAF_W, DG_LEAF_L, DG_NCOH_W, DG_NU2_W, DG_NU4_W,
       DG_NPRIM_L, DG_N };
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

// Per-phase instruction accounting (tools/isa_sections.py; never in the product). The lane
// loop is cut into regions at SEC(k):
//   FR_SEC_MARKS: SEC(k) is an assembler comment, so the ISA listing (hipcc -S) can be split
//                 into regions and each region's VALU instructions counted (static);
//   FR_SECCNT:    SEC(k) counts the wave-level entries of region k (first active lane, an LDS
//                 add; per launch into counters[4 + k]) (dynamic).
// Static VALU per region x wave entries per region = the launch's VALU instructions by phase.
// The first SC_N regions are counted; the others only mark a boundary in the listing, and
// their entries follow from a counted one (SETUP ~ CLAIM, ACC = NEED, POSTHIT = HIT,
// POSTSHADE = LATCH = ITER; GRAB = the batches the queue hands out).
// The BVH walk's node step and leaf tests each have a scalar path (every walking lane at one
// node or leaf) and a vector path, exclusive per entry: they are separate regions (SC_NODES /
// SC_NODEV, SC_LTESTS / SC_LTESTV), so a static count never adds both paths' instructions to
// one entry. SC_LIST: one primitive test of the compiled-in list loops (in a BVH kernel, the
// in-order fallback for far origins); SC_LROOT: a leaf sphere test's root step (discriminant
// > 0 on some lane). FR_SECCNT also sums the active lanes of every entry
// (counters[32 + k]).
enum { SC_ITER, SC_CLAIM, SC_JIT, SC_NEED, SC_REJ, SC_CAM, SC_SCAT, SC_HIT, SC_SKY, SC_SHADE, SC_END, SC_NODE,
       SC_LEAF, SC_NODES, SC_NODEV, SC_LTESTS, SC_LTESTV, SC_LIST, SC_LROOT, SC_N, SC_GRAB = SC_N, SC_SETUP, SC_ACC, SC_POSTHIT,
       SC_POSTSHADE, SC_LATCH, SC_NODET };
#if defined(FR_SEC_MARKS) && defined(__HIP_DEVICE_COMPILE__)
#define SEC(k) asm volatile(";FRSEC " #k)
#elif defined(FR_SECCNT)
#define SEC(k)                                                                       \
  do {                                                                               \
    const unsigned long long m_ = __ballot(1);                                       \
    if ((k) < SC_N && lane == static_cast<uint32_t>(__ffsll(m_) - 1)) {            \
      atomicAdd(&sec_cnt[(k) < SC_N ? (k) : 0], 1u);                               \
      atomicAdd(&sec_cnt[SC_N + ((k) < SC_N ? (k) : 0)], lanes_in(m_));            \
    }                                                                                \
  } while (0)
#else
#define SEC(k) do {} while (0)
#endif

// HAS_PLANE: planes may leave the shared record's t/p stale (plane.rs:27-29), so
// the last written t is tracked separately from the winner's.
// (two 32-bit popcounts: a 64-bit one leaves a 64-bit count whose compare the SALU
// cannot do, and the compiler moved it to the VALU)
// This lane's bit of a lane mask as its branch condition: LLVM's inverse ballot, which
// becomes the mask itself (an s_and_saveexec on it, no VALU). Declared by its intrinsic
// name: the hiprtc that builds the scene kernel (the one PyTorch ships) predates clang's
// __builtin_amdgcn_inverse_ballot_w64, its LLVM has the intrinsic.
extern "C" __device__ bool fr_inverse_ballot(unsigned long long) __asm("llvm.amdgcn.inverse.ballot.i64");
__device__ __forceinline__ bool lane_in(unsigned long long m) { return fr_inverse_ballot(m); }

__device__ __forceinline__ uint32_t lanes_in(unsigned long long m) {
  return static_cast<uint32_t>(__builtin_popcount(static_cast<uint32_t>(m)) +
                               __builtin_popcount(static_cast<uint32_t>(m >> 32)));
}
__device__ __forceinline__ uint32_t lanes_set(bool b) { return lanes_in(__builtin_amdgcn_ballot_w64(b)); }

// LDS byte address of a pointer into __shared__ memory, and the u32 at such an address
__device__ __forceinline__ uint32_t lds_addr(const uint32_t* p) {
  return static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) const uint32_t*)p));
}
__device__ __forceinline__ __attribute__((address_space(3))) uint32_t& lds_u32_at(uint32_t a) {
  return *reinterpret_cast<__attribute__((address_space(3))) uint32_t*>(static_cast<uintptr_t>(a));
}
// Per-lane select on a lane mask (a ballot): one v_cndmask_b32. The compiler turned chains
// of selects on compare results into branches with the conditions materialised as 0/1
// values in VGPRs; masks combined with SALU ops and this select keep them in SGPRs.
__device__ __forceinline__ uint32_t lane_sel(unsigned long long m, uint32_t if_set, uint32_t if_clear) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t r;
  asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r) : "v"(if_clear), "v"(if_set), "s"(m));
  return r;
#else
  return if_set;  // device only
#endif
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

#ifdef FR_JIT_N
#ifndef FR_JIT_GROUP
#define FR_JIT_GROUP 1024  // tests that may share terms (see the list walk; A/B knob)
#endif
#ifndef FR_JIT_PIN
#define FR_JIT_PIN 1  // settle the winner after every test (see the list walk; A/B knob)
#endif
// The scene-specialised build's records: FR_JIT_REC (jit.cpp) lists each primitive's 64-B
// device record as 16 u32 bit patterns (kind in word 15), so every float is exact,
// signed zeros and non-finite values included.
constexpr uint32_t kJitRec[FR_JIT_N][16] = {FR_JIT_REC};
template <uint32_t I>
struct JitRec {
  __device__ __forceinline__ float4 operator[](int k) const {
    return make_float4(__builtin_bit_cast(float, kJitRec[I][4 * k]), __builtin_bit_cast(float, kJitRec[I][4 * k + 1]),
                       __builtin_bit_cast(float, kJitRec[I][4 * k + 2]),
                       __builtin_bit_cast(float, kJitRec[I][4 * k + 3]));
  }
};
#endif

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
#ifndef FR_BVH_WAVES
// BVH kernels: 7 (72 VGPRs, one value spilled to scratch in the scatter step) over 6 (74
// VGPRs with the split scalar/vector node step): C5 trace 54.0 -> 51.4 ms
#define FR_BVH_WAVES 7
#endif
#define FR_OCC_ATTR                                                                                      \
  __attribute__((amdgpu_waves_per_eu(BVH ? FR_BVH_WAVES : DEFER == 2 ? FR_NIB_WAVES                   \
                                                      : (DEFER == 1 && MAT == 1) ? FR_DIFF12_WAVES : 7)))
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
#ifndef FR_TRACE_PRIO
#define FR_TRACE_PRIO 0
#endif
  // FR_TRACE_PRIO (A/B): the trace's waves issue ahead of a concurrently running sum_kernel
  // (the frame pipeline), which then only takes the issue slots the trace
  // leaves idle
  if (FR_TRACE_PRIO) __builtin_amdgcn_s_setprio(FR_TRACE_PRIO);
  extern __shared__ uint32_t lds[];
  constexpr bool NIB = DEFER == 2;             // 8-B records, winners in a register
  constexpr uint32_t STG = stage_samples(BVH, NIB);
  constexpr bool DIFFUSE = MAT == 1;           // lambertian scatters only
  constexpr bool SKYD = NIB && kSkyDefer;      // 12-B records {d.y, dot(d, d), winners}
  constexpr uint32_t WPS = NIB && !SKYD ? 2u : 3u;  // words per sample in the buffer
  // list kernels always stage; BVH kernels when the launch gave them the LDS (KF_STAGE)
  constexpr bool RSTG = BVH && FR_BVH_RSTAGE != 0;  // pairs staged in registers
  const bool staged = STG > 1 && !RSTG && (!BVH || NIB || (kp.flags & KF_STAGE) != 0u);
  float* stage = reinterpret_cast<float*>(lds) + threadIdx.x * (WPS * STG);
  // DEFER kernels (<= kDeferMaxPrims primitives) always hold the attenuations in LDS, and
  // the 8-B-record kernels (<= kNibbleMaxPrims) the records too: compile-time facts there,
  // so their global-load fallbacks are not compiled
  // (a BVH kernel with 8-B records stores attenuation classes, not primitive indices: its
  // scenes are larger than these tables)
  constexpr bool ATT_LDS = DEFER != 0 && !BVH, REC_LDS = NIB && !BVH;
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
  static_assert(!DEFER || (MAXD == 8 && !MT && (!BVH || (NIB && DIFFUSE))),
                "deferred unwind: depth <= 8 list kernels, or diffuse BVH kernels with 8-B records");
  uint2* drow = reinterpret_cast<uint2*>(stack) + tid;  // DEFER: this lane's 8 u8 levels
  uint8_t* bstack = reinterpret_cast<uint8_t*>(stack);
  uint4* hrow = reinterpret_cast<uint4*>(stack) + tid;  // this lane's MAXD = 8 levels
  // BVH traversal stack, after the unwind stack: kBvhStack x kBlock u32 (level-major)
  // (8-B-record kernels keep their winners in a register: no unwind stack in front)
  uint32_t* tstack = stack + (NIB ? 0u : MAXD ? (MAXD * kBlock) / 2u : (kp.max_depth ? kp.max_depth : 1u) * kBlock);
  // ... addressed by LDS byte address. Its first level is a sentinel row of kBvhEnd below
  // level 0, so that the top of an empty stack reads kBvhEnd: a pop needs no empty test.
  // tbase: level 0's first entry
  constexpr uint32_t kLevelB = 4u * kBlock;
  const uint32_t tbase = lds_addr(tstack) + kLevelB;
  if (BVH) tstack[tid] = kBvhEnd;  // (each lane reads only its own column)
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
#ifdef FR_SECCNT
  __shared__ uint32_t sec_cnt[2 * SC_N];  // wave entries, then active lanes summed over them
  if (tid < 2 * SC_N) sec_cnt[tid] = 0;
#endif
  __syncthreads();


  // NEED_JIT: a sample starts (its jitter, then its first lens try); NEED_LENS: a camera
  // lane's lens try after a rejected one
  enum : uint32_t { NEED_NONE = 0, NEED_LENS = 1, NEED_SPHERE = 2, NEED_JIT = 3 };
  uint32_t depth = 0;  // scatters of the path (not NIB: wnib holds them)
  // NIB: the winners as 4-bit entries, the last one pushed in bits 28..31 and the first in
  // bits 32 - 4 depth .. 35 - 4 depth, 15 on the levels below (empty). sum_kernel multiplies
  // nibble 7 first, so the path's winners are applied innermost first and the empty levels'
  // unit entries last (x * 1 = x). With d pushes nibble 8 - d is the first empty one:
  // depth < max_depth iff the nibbles under dmask are still empty.
  uint32_t wnib = ~0u;
  const uint32_t dmask = kp.max_depth ? (0xFu << (4u * (8u - min(kp.max_depth, 8u)))) : 0u;
  // stack push at level `depth` of the scatter winner
  auto push = [&](uint32_t pi) {
    if (NIB)
      wnib = (wnib >> 4) | (pi << 28);
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
  uint32_t sbest = 0, s = 0, s_end = 0, nseg = 0, nhit = 0;  // (scatters = segments - samples: the host's)
  // (a sample's index within its block is s mod kBlockSamples: blocks start at multiples of it)
  static_assert((kBlockSamples & (kBlockSamples - 1u)) == 0u, "blocks of a power-of-two sample count");
  V3 pend{0.0f, 0.0f, 0.0f};  // RSTG: the pair's first colour (an even jj)
#ifdef FR_DIAG
  uint32_t diag_tb = 0, diag_seg0 = 0;  // the item's batch index, segments at its claim
  uint32_t diag_iter = 0;               // loop iterations of this wave
#endif
  float* out = kw.samples;   // the item's first sample slot (item-major buffer)
  Rng rng{0u, 0u, 0u, 0u};
  // (a lane needs a work item when its block's samples are done: s == s_end, both 0 at the
  // start, and a claim that finds no pixel leaves them equal; a compare the loop's ballot
  // takes directly, where a carried bool cost a select and a compare per iteration)
  bool active = true, have_ray = false;
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
    SEC(SC_ITER);
    DIAG_WAVE(DG_ITER);
#ifdef FR_DIAG
    if (lane == 0 && (gw & 63u) == 0 && (gw >> 6) < 1024u && diag_iter < 1024u)
      g_fr_iter_times[(gw >> 6) * 1024u + diag_iter] = __builtin_amdgcn_s_memrealtime();
    ++diag_iter;
#endif
    const unsigned long long m = __builtin_amdgcn_ballot_w64(s == s_end);  // lanes needing an item
    // Lanes whose item is done wait (idle) until FR_CLAIM_MIN of them need one, or until no
    // active lane has other work: the claim step (its lane permutes and item setup) then
    // runs for several lanes at once instead of in nearly every iteration for one or two.
    // Only when work starts changes, never what a sample computes (results bit-identical).
    constexpr uint32_t CLAIM_MIN = NIB ? (BVH ? FR_CLAIM_MIN_BVH : FR_CLAIM_MIN_NIB) : FR_CLAIM_MIN;
    if (m && (CLAIM_MIN <= 1 || lanes_in(m) >= CLAIM_MIN || m == __ballot(1))) {
      SEC(SC_CLAIM);
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
        SEC(SC_GRAB);
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
      if (lane_in(m) && item >= kp.n_items) {
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
      if (lane_in(m)) {
        SEC(SC_SETUP);
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
          const uint32_t j0 = k * kFineSamples;
          s = (b & 0x0FFFFFFFu) * kBlockSamples + j0;
          out = kw.samples + WPS * (static_cast<size_t>(item - k * kp.P) * kp.ks);
#ifdef FR_DIAG
          diag_tb = item >> 6;
          diag_seg0 = nseg;
#endif
          s_end = min(s + (fine ? kFineSamples : kBlockSamples), kp.spp);
          // 2^24 x + 2^23, exact (x, yrow < 2^23): the jitter's numerator base (step 1)
          fx = static_cast<float>(x) * 16777216.0f + 8388608.0f;
          fy = static_cast<float>(yrow) * 16777216.0f + 8388608.0f;
          need = NEED_JIT;  // a sample starts: its jitter and lens sample in step 1
        }
      }
    }
    PROF_MARK(PF_CLAIM);
    bool ended = false;
    V3 term{0.0f, 0.0f, 0.0f};
    uint32_t tsky = kDeferAbsorbed;  // DEFER: the terminal as sky parameter bits (SKYD: dot(d, d))
    float sky_dy = 0.0f;             // SKYD: the escaping ray's d.y
    if (need != NEED_NONE) {
      SEC(SC_NEED);
      // 1. merged rejection loop
      // mrej: the lanes that still reject (dd >= 2^46), one compare per pass: the loop test
      // counts it and the next pass's branch and the accept test take it back as their
      // lane condition (inverse ballot, no instruction; a compare on dd in each of them
      // cost the pass a second v_cmp, a bool carried through the loop a select and a compare).
      // Every lane here makes the first try, outside the loop: px, py and dd need no
      // initial values then
      // (the sphere/circle condition as a lane mask: one compare serves the tries and the
      // camera/scatter branch, which the compiler otherwise tested with a second v_cmp)
      const unsigned long long msph = __builtin_amdgcn_ballot_w64(need == NEED_SPHERE);
      float pz = 0.0f;  // a circle try keeps pz = 0
      DIAG_WAVE(DG_LENS_W);
      DIAG_LANE(DG_LENS_L);
      // the test in the 2^23-scaled domain (rng_signed_unit_scaled): same decisions
      float px = rng_signed_unit_scaled(rng);
      float py = rng_signed_unit_scaled(rng);
      // A sample's first draws are its jitter (tracer.rs:171-172), then its lens try: a
      // starting lane's first try takes four draws where a scatter lane's takes three (and a
      // camera lane's retry two). The third draw is made by both kinds in one instruction
      // sequence; a starting lane's first two are its jitter and it draws its try's fourth
      // in the branch below (the jitter's own two draws in their own branch, in the quarter
      // of lanes that start a sample, cost a branch of 31 VALU)
      const unsigned long long mjit = __builtin_amdgcn_ballot_w64(need == NEED_JIT);
      float pw = 0.0f;
      if (lane_in(msph | mjit)) pw = rng_signed_unit_scaled(rng);
      if (lane_in(msph)) pz = pw;
      if (lane_in(mjit)) {
        SEC(SC_JIT);
        // 2^24 r = (int32)u >> 8 + 2^23 (rng_f32_scaled; exact), so 2^24 x + 2^24 r =
        // (2^24 x + 2^23) + px, one rounding either way. 2^24 (x + r) = RN(2^24 x + 2^24 r)
        // (rounding commutes with the exact scaling), so the quotients are (x + r) / W's
        // bits: numerator +0 or in [1, 2^56], divisor 2^24 W
        d.x = div_rn(fx + px, kp.sW, kp.rW);
        d.y = div_rn(fy + py, kp.sH, kp.rH);
        if (MT) d.y = d.y + vofs;  // render_mt's band offset (tracer.rs:103)
        px = pw;
        py = rng_signed_unit_scaled(rng);
        need = NEED_LENS;
      }
      float dd = px * px + py * py + pz * pz;
      unsigned long long mrej = __builtin_amdgcn_ballot_w64(dd >= kUnitBallScaled);
      while (lanes_in(mrej) > static_cast<uint32_t>(KREJ)) {
        SEC(SC_REJ);
        DIAG_WAVE(DG_LENS_W);
        DIAG_LANE(DG_LENS_L);
        if (lane_in(mrej)) {
          px = rng_signed_unit_scaled(rng);
          py = rng_signed_unit_scaled(rng);
          if (lane_in(msph)) pz = rng_signed_unit_scaled(rng);
          dd = px * px + py * py + pz * pz;
        }
        mrej = __builtin_amdgcn_ballot_w64(dd >= kUnitBallScaled);
      }
      SEC(SC_ACC);
      if (!lane_in(mrej)) {
        // the accepted point is k 2^-23 per coordinate (2r - 1, exact), k = (px, py, pz):
        // the scale is folded into the operation that uses it (below)
        if (!lane_in(msph)) {
          SEC(SC_CAM);
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
          // lens * (k 2^-23) = (lens 2^-23) * k when lens 2^-23 is exact (KCam::lens_pre):
          // the same product, one rounding
          const V3 rd = cm.lens_pre ? V3{cm.lens_s * px, cm.lens_s * py, 0.0f}
                                    : scl(cm.lens, V3{px * kSignedUnitScale, py * kSignedUnitScale, 0.0f});
          const V3 off = add(scl(rd.x, cu), scl(rd.y, cv));
          const float u = d.x, v = d.y;
          o = add(cpos, off);
          d = sub(sub(add(add(cllc, scl(u, chor)), scl(v, cver)), cpos), off);
          if (!NIB) depth = 0;
          have_ray = true;
        } else {
          SEC(SC_SCAT);
          bool ok = true;
          V3 dir;
          if (!DIFFUSE && smetal) {
            const V3 r{px * kSignedUnitScale, py * kSignedUnitScale, pz * kSignedUnitScale};
            dir = add(d, scl(sfuzz, r));  // reflected + fuzz * rus
            ok = dot(dir, sn) > 0.0f;     // sphere.rs:104 / plane.rs:121
          } else {
            // ((p + n) + rus) - p; p + n + k 2^-23 as one fma (the product is exact)
            const V3 dr{__builtin_fmaf(px, kSignedUnitScale, d.x), __builtin_fmaf(py, kSignedUnitScale, d.y),
                        __builtin_fmaf(pz, kSignedUnitScale, d.z)};
            dir = sub(dr, o);
          }
          if (ok) {
            if (!(NIB && DIFFUSE)) push(sbest);  // (NIB && DIFFUSE kernels pushed at the shading step)
            if (!NIB) ++depth;
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
      SEC(SC_HIT);
      // 2. closest hit over the list in order (tracer.rs:190-200): only the accepted t
      // of each test is needed here; the record is formed for the winner below.
      ++nseg;
      V3 inv{recip_nr(d.x), recip_nr(d.y), recip_nr(d.z)};
      // (non-short-circuit: one branch to the rare fallback instead of three nested ones)
      // FR_BOX_FMA: the box test's reciprocal is RN(1 / d) clamped to +-2^100 (rt_core.h
      // box_inv): recip_nr's range is narrowed to |d| >= 2^-100, where the clamp is the
      // identity, and the fallback clamps
      const int rok = FR_BOX_FMA ? static_cast<int>(recip_box_ok(d.x)) & static_cast<int>(recip_box_ok(d.y)) &
                                       static_cast<int>(recip_box_ok(d.z))
                                 : static_cast<int>(recip_nr_ok(d.x)) & static_cast<int>(recip_nr_ok(d.y)) &
                                       static_cast<int>(recip_nr_ok(d.z));
      if (!rok) {
        inv = V3{1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
        if (FR_BOX_FMA) inv = V3{box_inv_clamp(inv.x), box_inv_clamp(inv.y), box_inv_clamp(inv.z)};
      }
      const V3 boinv{o.x * inv.x, o.y * inv.y, o.z * inv.z};  // (FR_BOX_FMA box tests only)
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
        // (DESIGN.md §4.7). A lane steps into the nearer entered child and stacks the
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
          // this lane's next free traversal-stack entry as its LDS byte address (level-major:
          // one level is kBlock entries, kLevelB bytes); the stack is empty while it is in
          // level 0, and the entry below it is the sentinel row. (As an index, every read and
          // write cost an address add.)
          uint32_t tso = tbase + 4u * tid;
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
              SEC(SC_NODE);
              DIAG_WAVE(DG_NODE_W);
              DIAG_LANE(DG_NODE_L);
#ifdef FR_DIAG
              {
                // distinct nodes among the walking lanes (1, 2, 3-4, more), and lanes of primary rays
                unsigned long long m_ = __ballot(1);
                uint32_t u_ = 0;
                while (m_ && u_ < 5) {
                  const uint32_t r_ = __builtin_amdgcn_readlane(ref, __ffsll(m_) - 1);
                  m_ &= ~__ballot(ref == r_);
                  ++u_;
                }
                if (u_ == 1) DIAG_WAVE(DG_NCOH_W);
                if (u_ == 2) DIAG_WAVE(DG_NU2_W);
                if (u_ == 3 || u_ == 4) DIAG_WAVE(DG_NU4_W);
                if (depth == 0) DIAG_LANE(DG_NPRIM_L);
              }
#endif
              // the stack's top, read before the node arrives (the sentinel kBvhEnd when the
              // stack is empty)
              typedef unsigned long long Mask;  // lane masks (ballots of single compares)
              const uint32_t tdown = tso - kLevelB;
              const uint32_t top = lds_u32_at(tdown);
              // the step's outcome, applied after the scalar or vector path (each path doing it
              // itself left a register copy of the stack position at the loop's latch)
              uint32_t t_near, t_far;
              Mask t_many, t_both;
              // internal node: both children's boxes; the nearer entered child next (the
              // left one on a tie) and the other stacked when both are entered; neither: the
              // stack's top (the sentinel ends the walk). Branch-free: the far child is written
              // to the free entry either way (a node at depth d has at most d entries below it,
              // d < kBvhStack) and the index moves only on a push or pop. (A ballot of an & of
              // compares went through a 0/1 VGPR and a compare: the compares' own masks are
              // combined with SALU ops.)
              auto node_pick = [&](const Slab& sl, const Slab& sr, const uint32_t cl, const uint32_t cr) {
                const Mask ml = __builtin_amdgcn_ballot_w64(sl.tn <= sl.tf) &
                                __builtin_amdgcn_ballot_w64(sl.tf >= 0.001f) & __builtin_amdgcn_ballot_w64(sl.tn <= closest);
                const Mask mr = __builtin_amdgcn_ballot_w64(sr.tn <= sr.tf) &
                                __builtin_amdgcn_ballot_w64(sr.tf >= 0.001f) & __builtin_amdgcn_ballot_w64(sr.tn <= closest);
                const Mask mgol = ml & (__builtin_amdgcn_ballot_w64(sl.tn <= sr.tn) | ~mr);
                const Mask many = ml | mr;
                // near = mgol ? cl : cr and far = the other, as xors with cl ^ cr: in the scalar
                // step cl and cr are SGPRs, and a select between two SGPRs needs one of them
                // copied to a VGPR first (one scalar operand per VALU instruction)
                const uint32_t cx = cl ^ cr;
                const uint32_t near = cl ^ lane_sel(mgol, 0u, cx);
                t_near = near;
                t_far = near ^ cx;
                t_many = many;
                t_both = ml & mr;
              };
              auto node_step = [&](const float4 na, const float4 nb, const float4 nc, const uint32_t cl,
                                   const uint32_t cr) {
                node_pick(slab3_fused(xyz(na), xyz(nb), oinv, invc),
                          slab3_fused(V3{na.w, nc.x, nc.y}, V3{nb.w, nc.z, nc.w}, oinv, invc), cl, cr);
              };
#if FR_BVH_SCALAR_NODES
              const uint32_t ref0 = __builtin_amdgcn_readfirstlane(ref);
              if (__ballot(ref != ref0) == 0) {
                // every walking lane is at the same node (90 % of C5's node steps): scalar
                // loads, the slab arithmetic on SGPR operands (the distinct asm ends keep the
                // two paths from being merged over copies of the node into VGPRs)
                const RecRef nd = rec_at(sc.bvh, ref0);
                const float4 r = nd[3];
                SEC(SC_NODES);
                node_step(nd[0], nd[1], nd[2], __float_as_uint(r.x), __float_as_uint(r.y));
                asm volatile("; bvh node step: scalar");
              } else
#endif
              {
                SEC(SC_NODEV);
                const uint32_t nb0 = ref * 64u;  // node byte offset (< 2^32: nodes < 2^26)
                const uint4 nr = __builtin_bit_cast(uint4, buf_load4(sc.bvh, nb0 + 48u));
                node_step(buf_load4(sc.bvh, nb0), buf_load4(sc.bvh, nb0 + 16u), buf_load4(sc.bvh, nb0 + 32u), nr.x, nr.y);
                asm volatile("; bvh node step: vector");
              }
              SEC(SC_NODET);
              lds_u32_at(tso) = t_far;  // the far child
              const uint32_t tpop = lane_sel(t_many, tso, tdown);
              ref = lane_sel(t_many, t_near, top);
              tso = lane_sel(t_both, tso + kLevelB, tpop);
            }
            if (ref == kBvhEnd) break;
            SEC(SC_LEAF);
            DIAG_WAVE(DG_LEAF_W);
            DIAG_LANE(DG_LEAF_L);
            // leaf: slots [first, first + count) of the leaf-order records; one test of
            // primitive i (list index) whose leaf-order record r is at `slot`
            auto leaf_test = [&](const uint32_t i, const auto& r) {
              const float tmax =
                  static_cast<int>(i) < best ? __uint_as_float(__float_as_uint(closest) + 1u) : closest;
              const uint32_t k = KS == KS_AABB ? FR_AABB : KS == KS_SPHERE ? FR_SPHERE : __float_as_uint(r[3].w);
              float t = 0.0f;
              bool h = false;
              if (k == FR_SPHERE) {
                const float4 g = r[0];  // centre, RN(radius^2) (the leaf records' form)
#ifndef FR_SPHERE_IEEE
                const SphereDisc q = sphere_disc_rr(xyz(g), g.w, o, d, a_dd);
                if (q.disc > 0.0f) {
                  SEC(SC_LROOT);
                  h = sphere_roots_fast(q, a_dd, ssg, 0.001f, tmax, t);
                }
#else
                h = sphere_root_rr(xyz(g), g.w, o, d, a_dd, 0.001f, tmax, t);
#endif
              } else if (k == FR_AABB) {
                h = slab_root(slab3_box(xyz(r[0]), xyz(r[1]), o, inv, boinv), 0.001f, tmax, t);
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
            };
            const uint32_t first = ref & ((1u << kBvhSlotBits) - 1u);
            const uint32_t cnt = ((ref >> kBvhSlotBits) & 15u) + 1u;
#if FR_BVH_SCALAR_LEAVES
            const uint32_t leaf0 = __builtin_amdgcn_readfirstlane(ref);
            if (__ballot(ref != leaf0) == 0) {
              // every lane at one leaf: its records through scalar loads
              typedef __attribute__((address_space(4))) const uint32_t cu32l;
              const cu32l* ord = (cu32l*)(reinterpret_cast<uintptr_t>(sc.bvh_order));
              const uint32_t first0 = leaf0 & ((1u << kBvhSlotBits) - 1u);
              const uint32_t cnt0 = ((leaf0 >> kBvhSlotBits) & 15u) + 1u;
              for (uint32_t kk = 0; kk < cnt0; ++kk) {
                SEC(SC_LTESTS);
                leaf_test(ord[first0 + kk], rec_at(sc.lrec, first0 + kk));
              }
              asm volatile("; bvh leaf: scalar");
            } else
#endif
            {
              for (uint32_t kk = 0; kk < cnt; ++kk) {
                SEC(SC_LTESTV);
                const uint32_t slot = first + kk;
                // buffer loads: 32-bit offsets from the arrays' bases (slots < 2^26)
                struct LeafRec {
                  const float4* base;
                  uint32_t off;
                  __device__ float4 operator[](uint32_t k) const { return buf_load4(base, off + 16u * k); }
                } const r{sc.lrec, slot * 64u};
                leaf_test(buf_load1(sc.bvh_order, slot * 4u), r);
              }
              asm volatile("; bvh leaf: vector");
            }
            tso -= kLevelB;  // pop (the sentinel kBvhEnd when the stack was empty)
            ref = lds_u32_at(tso);
          }
        }
      }
      // one primitive of kind K at list index i (wave-uniform), its record read through r4:
      // scalar loads (RecRef), or compile-time constants in the scene-specialised build
      auto test_rec = [&](auto kind_tag, uint32_t i, const auto& r4) {
        constexpr uint32_t K = decltype(kind_tag)::value;
        float t = 0.0f;
        bool h = false;
        if constexpr (K == FR_AABB) {
          h = slab_root(slab3_box(xyz(r4[0]), xyz(r4[1]), o, inv, boinv), 0.001f, closest, t);
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
#if defined(FR_JIT_N) && defined(__HIP_DEVICE_COMPILE__)
        // scene-specialised list: the winner (and the last written t) settled after every
        // test; otherwise the compiler sinks the chain of selects into the shading step and
        // keeps every test's hit mask and t live until then (a 43-primitive list spilled
        // 64 SGPRs and 62 VGPRs)
        if constexpr (FR_JIT_PIN && !std::is_same<typename std::decay<decltype(r4)>::type, RecRef>::value) {
          asm volatile("" : "+v"(best));
          if (HAS_PLANE) asm volatile("" : "+v"(t_last));
        }
#endif
      };
      auto test_one = [&](auto kind_tag, uint32_t i) {
        SEC(SC_LIST);
        test_rec(kind_tag, i, rec_at(sc.rec, i));
      };
      typedef std::integral_constant<uint32_t, FR_AABB> TagAabb;
      typedef std::integral_constant<uint32_t, FR_SPHERE> TagSphere;
#ifdef FR_JIT_N
      if constexpr (!BVH) {
        // Scene-specialised build (jit.cpp): the list in order, unrolled, every record a
        // compile-time constant. The tests and their order are the list loop's, so the
        // results are the same bits; what changes is that slab distances and other terms
        // two primitives share (a coordinate plane common to several boxes) are computed
        // once per segment, and no record is loaded.
        auto test_j = [&](auto ic) {
          constexpr uint32_t I = decltype(ic)::value;
          constexpr uint32_t K = kJitRec[I][15];
#if defined(__HIP_DEVICE_COMPILE__)
          // Every FR_JIT_GROUP tests, the ray passes through an empty asm: later tests
          // compute from new (equal) values, so terms are shared only within a group. A
          // shared term is held in a register until its last use; across a 43-primitive
          // list that spilled 62 VGPRs.
          if constexpr (I > 0 && I % FR_JIT_GROUP == 0)
            asm volatile("" : "+v"(o.x), "+v"(o.y), "+v"(o.z), "+v"(d.x), "+v"(d.y), "+v"(d.z), "+v"(inv.x),
                         "+v"(inv.y), "+v"(inv.z));
#endif
          if constexpr (K == FR_AABB || K == FR_SPHERE || K == FR_PLANE || K == FR_TRIANGLE || K == FR_OBB) {
            test_rec(std::integral_constant<uint32_t, K>{}, I, JitRec<I>{});
          }
          // FR_STUB: never hits (aabb.rs:21-34, rectangle.rs:21-34)
        };
        unroll_below<0u, FR_JIT_N>(FR_JIT_N, test_j);
      } else
#endif
#ifndef FR_NO_UNROLL_NIB
      if constexpr (NIB && !BVH && KS != KS_ANY) {
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
      SEC(SC_POSTHIT);
      if (best < 0) {
        SEC(SC_SKY);
        if (SKYD) {
          sky_dy = d.y;
          tsky = __float_as_uint(d.x * d.x + d.y * d.y + d.z * d.z);  // length()'s sum, in its order
        } else if (DEFER)
#ifndef FR_SKY_IEEE
          // the sqrt and division by their core sequences under a range guard (sky_t_fast,
          // bit-identical): C3 frame 15.52 -> 15.27 ms (in round 3, before the sum ran beside
          // the trace, it had measured neutral); FR_SKY_IEEE builds the compiler's sequences
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
        if (NIB ? (dmask != 0u && (wnib & dmask) == dmask) : depth < kp.max_depth) {
          SEC(SC_SHADE);
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
            n = slab_normal(slab3_box(xyz(b0), xyz(b1), o, inv, boinv), closest, d);
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
          // a lambertian scatter always continues the path (sphere.rs:84-89): with only those
          // (and stubs, which end it above) the winner is pushed here, not held to the scatter
          if (NIB && DIFFUSE && c != SC_NONE) {
            if (BVH)
              push(buf_load1(sc.acls, 4u * static_cast<uint32_t>(best)));  // the winner's attenuation class
            else
              push(static_cast<uint32_t>(best));
          }
          if (!DIFFUSE && c == SC_DIELECTRIC) {
            // one draw, no rejection loop (sphere.rs:107-145)
            d = scatter_dielectric(din, n, rng);
            push(static_cast<uint32_t>(best));
            if (!NIB) ++depth;
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
    SEC(SC_POSTSHADE);
    if (ended) {
      SEC(SC_END);
      // 3. attenuation * get_color(...) (tracer.rs:206-207), innermost first
      DIAG_WAVE(DG_END_W);
      DIAG_LANE(DG_END_L);
      V3 col = term;
      if (SKYD) {
        col = V3{sky_dy, __uint_as_float(tsky), __uint_as_float(wnib)};
        wnib = ~0u;  // the next sample starts empty
      } else if (NIB) {
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
      const uint32_t jj = s & (kBlockSamples - 1u);  // the sample's index in its block
      if (RSTG) {
        // pairs start on even jj (blocks and sub-blocks do): the odd sample stores both
        if (jj & 1u) {
          float* dst = out + WPS * (jj - 1u);
          if (kp.ks == kBlockSamples) {
            if constexpr (WPS == 3u) {
              // 8-B aligned: item * 192 B + a multiple of 24 B
              reinterpret_cast<float2*>(dst)[0] = make_float2(pend.x, pend.y);
              reinterpret_cast<float2*>(dst)[1] = make_float2(pend.z, col.x);
              reinterpret_cast<float2*>(dst)[2] = make_float2(col.y, col.z);
            } else {
              // 16-B aligned: item * 128 B + a multiple of 16 B
              *reinterpret_cast<float4*>(dst) = make_float4(pend.x, pend.y, col.x, col.y);
            }
          } else {
            dst[0] = pend.x;
            dst[1] = pend.y;
            if (WPS == 3) dst[2] = pend.z;
            dst[WPS] = col.x;
            dst[WPS + 1] = col.y;
            if (WPS == 3) dst[WPS + 2] = col.z;
          }
        } else if (s + 1u == s_end) {
          out[WPS * jj] = col.x;
          out[WPS * jj + 1] = col.y;
          if (WPS == 3) out[WPS * jj + 2] = col.z;
        } else {
          pend = col;
        }
      } else if (!staged) {
        out[WPS * jj] = col.x;
        out[WPS * jj + 1] = col.y;
        if (WPS == 3) out[WPS * jj + 2] = col.z;
      } else {
        // stage the colour; every STG-th sample of the block, and its last, go out together.
        // FR_STAGE_SMAJOR (8-B records): slot-major staging, slot j of every lane of the
        // workgroup contiguous (a wave's writes conflict-free) instead of each lane's
        // STG slots contiguous (lanes 8 apart on one bank)
        constexpr bool SMAJ = FR_STAGE_SMAJOR != 0 && WPS == 2u && STG == 4u;
        float* const stage_base = reinterpret_cast<float*>(lds);
        auto slot_at = [&](uint32_t js) -> float* {
          return SMAJ ? stage_base + (js * kBlock + tid) * WPS : stage + WPS * js;
        };
        float* sl = slot_at(jj & (STG - 1u));
        sl[0] = col.x;
        sl[1] = col.y;
        if (WPS == 3) sl[2] = col.z;
        const bool full = (jj & (STG - 1u)) == STG - 1u;
        if (full || s + 1u == s_end) {
          const uint32_t g0 = jj & ~(STG - 1u);
          // (a sub-block inside a wider group stores from its own first sample)
          // (its first sample: items of block b_fine are the 4-aligned sub-blocks, derived
          // here rather than held in a register through the loop)
          const bool fine_item = kStageSpansSub && kp.b_fine != 0u && s / kBlockSamples == kp.b_fine;
          const uint32_t lo = fine_item ? (jj & ~(kFineSamples - 1u)) : g0;
          float* dst = out + WPS * g0;
          if (full && kp.ks == kBlockSamples && lo == g0) {
            if constexpr (SMAJ) {
              // two slots per 16-B store
              const float2 a0 = *reinterpret_cast<const float2*>(slot_at(0)), a1 = *reinterpret_cast<const float2*>(slot_at(1));
              const float2 a2 = *reinterpret_cast<const float2*>(slot_at(2)), a3 = *reinterpret_cast<const float2*>(slot_at(3));
              reinterpret_cast<float4*>(dst)[0] = make_float4(a0.x, a0.y, a1.x, a1.y);
              reinterpret_cast<float4*>(dst)[1] = make_float4(a2.x, a2.y, a3.x, a3.y);
            } else if constexpr ((WPS * STG) % 4u == 0u) {
              // 16-B aligned: item * 192 (128) B + a multiple of 48 (32) B
              const float4* src = reinterpret_cast<const float4*>(stage);
#pragma unroll
              for (uint32_t k = 0; k < WPS * STG / 4u; ++k) {
                reinterpret_cast<float4*>(dst)[k] = src[k];
#if defined(__HIP_DEVICE_COMPILE__)
                // wide groups: two 16-B stores at a time, not every LDS read first (registers)
                if (WPS * STG > 8u) asm volatile("" ::: "memory");
#endif
              }
            } else {
              // 8-B aligned: item * 192 B + a multiple of 24 B
              const float2* src = reinterpret_cast<const float2*>(stage);
#pragma unroll
              for (uint32_t k = 0; k < WPS * STG / 2u; ++k) reinterpret_cast<float2*>(dst)[k] = src[k];
            }
          } else {
            for (uint32_t k = WPS * (lo - g0); k < WPS * ((jj & (STG - 1u)) + 1u); ++k)
              dst[k] = SMAJ ? slot_at(k / WPS)[k % WPS] : stage[k];
          }
        }
      }
#ifdef FR_DIAG
      if (s + 1u == s_end && diag_tb < (1u << 20)) atomicAdd(&g_fr_tb_cost[diag_tb], nseg - diag_seg0);
#endif
      if (++s != s_end) need = NEED_JIT;  // next sample of the block, same stream (else: a new item)
    }
    PROF_MARK(PF_END);
    SEC(SC_LATCH);
  }

  // Per-wave counter reduction into the wave's own slot (plain stores): the waves leave
  // the drain within a fraction of a millisecond, and three returning atomics per wave on
  // one cache line queued long enough there to hold the kernel's end back.
  unsigned long long a = nseg, b = nhit, sct = 0;
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
#ifdef FR_SECCNT
  __syncthreads();
  if (tid < SC_N) atomicAdd(&kw.counters[4 + tid], static_cast<unsigned long long>(sec_cnt[tid]));
  if (tid < SC_N) atomicAdd(&kw.counters[32 + tid], static_cast<unsigned long long>(sec_cnt[SC_N + tid]));
#endif
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

}  // namespace fr
