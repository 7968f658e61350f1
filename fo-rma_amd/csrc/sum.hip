// sum.hip — sum_kernel: adds each pixel's sample records of a pass, in sample order,
// onto its running sum, and at the last pass divides, gamma-corrects and quantises
// (tracer.rs:170-184). Launched by render.hip through launch_sum (sum.h).
#include "sum.h"

namespace fr {

#ifndef FR_SUM_UNROLL
#define FR_SUM_UNROLL 2
#endif
constexpr int kSumUnroll = FR_SUM_UNROLL;
#ifndef FR_SUM_UNROLL_SKYD
#define FR_SUM_UNROLL_SKYD 1
#endif
constexpr int kSumUnrollSkyd = FR_SUM_UNROLL_SKYD;
static_assert(kSumThreads % 64u == 0 && kSumThreads <= kDeferUnit + 1u, "whole waves, one table pass or more");

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

// FR_SUM_VGPR_CAP: the sum runs beside seven trace workgroups per CU,
// whose 56 VGPRs per wave leave 120 per SIMD lane for one sum wave
#ifndef FR_SUM_VGPRS
#define FR_SUM_VGPRS 120
#endif
#if FR_SUM_VGPRS
#define FR_SUM_VGPR_CAP __attribute__((amdgpu_num_vgpr(FR_SUM_VGPRS)))
#else
#define FR_SUM_VGPR_CAP
#endif
// KIND 1: FR_SKY_DEFER's 12-B records only (a kernel without the other paths' registers)
template <uint32_t WPS, int KIND = 0>
__global__ __launch_bounds__(kSumThreads) FR_SUM_VGPR_CAP void sum_kernel(KParams kp, const float* __restrict__ samples,
                                                          float* __restrict__ running, float* __restrict__ out_mean,
                                                          uint8_t* __restrict__ out_u8, int first, int last,
                                                          const float4* __restrict__ att, uint32_t n_prims) {
  constexpr uint32_t kSumSlot = WPS * kBlockSamples + 1;  // floats per slot in LDS (odd stride)
  constexpr int kUnroll = KIND == 1 ? kSumUnrollSkyd : kSumUnroll;
  // one LDS block, the attenuation table first: its entries then sit at LDS byte offset
  // 12 x index, and the per-level reads need no base-address add (the table behind the
  // tile, at 33,792 B, cost a v_or per level: 8 of ~60 VALU per sample)
  // 8-B records (WPS 2) read a 16-B-stride copy of the first 16 entries: level k's byte
  // offset is then one shift-and-mask of the winners word (below)
  constexpr uint32_t kTable = 4u * 16u + 3u * (kDeferUnit + 1u);  // floats
  __shared__ float lds_sum[kTable + kSumThreads * kSumSlot];
  float4* const att16 = reinterpret_cast<float4*>(lds_sum);
  float* const att_s = lds_sum + 4 * 16;  // KF_DEFER: attenuation rgb, entry kDeferUnit = 1
  float* const tile = lds_sum + kTable;
#ifndef FR_SUM_PRIO
#define FR_SUM_PRIO 0
#endif
  // Pipelined frames run this kernel on the CU slot the next frame's
  // trace leaves free, where it takes about as long as the trace. A raised wave priority
  // slowed the trace by more than it sped the sum (FR_SUM_PRIO=3: C3 streamed 16.65 ->
  // 17.07 ms per frame in round 3; 1: 16.26 -> 16.73 in round 4): not used.
  if (FR_SUM_PRIO) __builtin_amdgcn_s_setprio(FR_SUM_PRIO);
#ifdef FR_SUM_STUB
  return;  // measurement-only builds (tools/stream_ab.py --allow-diff): the frame without its sum
#endif
  const uint32_t t = threadIdx.x;
  const bool defer = (kp.flags & KF_DEFER) != 0;
  if (defer) {  // the kDeferUnit + 1 table entries, kSumThreads at a time
    for (uint32_t i = t; i <= kDeferUnit; i += kSumThreads) {
      const float4 a = i < n_prims ? att[i] : make_float4(1.0f, 1.0f, 1.0f, 0.0f);
      att_s[3 * i] = a.x;
      att_s[3 * i + 1] = a.y;
      att_s[3 * i + 2] = a.z;
      if (i < 16u) att16[i] = make_float4(a.x, a.y, a.z, 0.0f);
    }
  }
  const uint32_t q0 = blockIdx.x * kSumThreads, q = q0 + t;
  const uint32_t nq = min(kSumThreads, kp.P - q0);
  uint32_t x = 0, y = 0;
  const bool valid = q < kp.P && slot_xy(kp, q, x, y);
  const bool mt = (kp.flags & FR_FLAG_MT_BANDS) != 0;
  const bool mt_zero = mt && !(kp.band_h && y / kp.band_h < 4u);  // rows render_mt never fills stay 0
  V3 sum = (first || !valid) ? V3{0.0f, 0.0f, 0.0f} : V3{running[3 * q], running[3 * q + 1], running[3 * q + 2]};
#ifndef FR_SUM_BUFLOAD
#define FR_SUM_BUFLOAD 1
#endif
#ifndef FR_SUM_WAITFIX
#define FR_SUM_WAITFIX 1
#endif
  // The running sum's loads land here, before the first block's loads are issued. Left to
  // the compiler, the wait for them sat on the first add of every block's sample loop,
  // where (global loads complete in order) it also waited for the next block's prefetch.
  if (FR_SUM_WAITFIX) asm volatile("" : "+v"(sum.x), "+v"(sum.y), "+v"(sum.z));
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
    if (FR_SUM_BUFLOAD) {
      // buffer loads: a 32-bit lane offset per load instead of a 64-bit address; the
      // descriptor's range (the workgroup's n4 float4) returns 0 past the last slot. The
      // whole offset is in the lane operand: the raw-buffer range check covers the lane
      // offset, and the scalar offset may be outside it on this family
      const __amdgpu_buffer_rsrc_t r =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float4*>(src4), 0, static_cast<int>(n4 * 16u), 0x00020000);
      typedef float v4f __attribute__((ext_vector_type(4)));
#pragma unroll
      for (uint32_t k = 0; k < kV; ++k) {
        const v4f x = __builtin_amdgcn_raw_buffer_load_b128(r, t * 16u + k * kSumThreads * 16u, 0, 0);
        v[k] = make_float4(x.x, x.y, x.z, x.w);
      }
      return;
    }
#pragma unroll
    for (uint32_t k = 0; k < kV; ++k) {
      const uint32_t i = t + k * kSumThreads;
      if (FR_SUM_WAITFIX) {
        // every lane loads (past the last slot: the last float4 again), so the loads and
        // the tile stores below are straight-line code: the wait before each store is for
        // its own load, and no load waits for the one before it
        v[k] = src4[min(i, n4 - 1u)];
      } else if (i < n4) {
        v[k] = src4[i];
      }
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
        if (FR_SUM_WAITFIX || i < n4) {  // (slots past nq are never read)
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
      // FR_SUM_UNROLL: samples whose colour rebuilds interleave (the sums stay in order)
#pragma unroll kUnroll
      for (uint32_t j = 0; j < n; ++j, c += WPS) {
        if (WPS == 2 && KIND == 0) {
          // 8-B record: terminal, then a_7 ... a_0 from 4-bit entries (kNibbleUnit: 1)
          const uint32_t tb = __float_as_uint(c[0]), w = __float_as_uint(c[1]);
          V3 col = tb == kDeferAbsorbed ? V3{0.0f, 0.0f, 0.0f} : sky_from_t(c[0]);
          // level k's entry at byte 16 x nibble k: odd levels are the high nibble of byte
          // k / 2 of w, even levels the high nibble of byte k / 2 of w << 4
          const uint32_t w4 = w << 4;
#pragma unroll
          for (int k = 7; k >= 0; --k) {
            const uint32_t off = (((k & 1) ? w : w4) >> (8 * (k >> 1))) & 0xF0u;
            const float4 e = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(att16) + off);
            col = mul(V3{e.x, e.y, e.z}, col);
          }
          sum = add(sum, col);
        } else if (KIND == 1 || (kSkyDefer && (kp.flags & KF_NIBBLE))) {
          // FR_SKY_DEFER's 12-B record {d.y, dot(d, d), winners}: the sky parameter here
          const float dd = c[1];
          const uint32_t w = __float_as_uint(c[2]);
#ifdef FR_SKY_SUM_IEEE
          const float tt = sky_t_from(c[0], dd);
#else
          const float tt = sky_t_fast_from(c[0], dd);  // bit-identical (fr_selftest_ops op 14)
#endif
          V3 col = __float_as_uint(dd) == kDeferAbsorbed ? V3{0.0f, 0.0f, 0.0f} : sky_from_t(tt);
          const uint32_t w4 = w << 4;
#pragma unroll
          for (int k = 7; k >= 0; --k) {
            const uint32_t off = (((k & 1) ? w : w4) >> (8 * (k >> 1))) & 0xF0u;
            const float4 e = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(att16) + off);
            col = mul(V3{e.x, e.y, e.z}, col);
          }
          sum = add(sum, col);
        } else if (KIND == 0 && defer) {
          // the deferred unwind (kDeferUnit): terminal, then a_7 ... a_0 innermost first
          const uint32_t tb = __float_as_uint(c[0]), lo = __float_as_uint(c[1]), hi = __float_as_uint(c[2]);
          V3 col = tb == kDeferAbsorbed ? V3{0.0f, 0.0f, 0.0f} : sky_from_t(c[0]);
#pragma unroll
          for (int k = 7; k >= 0; --k) {
            const float* e = att_s + 3u * (((k >= 4 ? hi : lo) >> (8 * (k & 3))) & 0xFFu);
            col = mul(V3{e[0], e[1], e[2]}, col);
          }
          sum = add(sum, col);
        } else if (KIND == 0 && mt) {  // save_image_mt (tracer.rs:140-145): acc += (sqrt(c) * 255) as u8 / sample
          sum = add(sum, V3{static_cast<float>(to_u8(c[0])) / fspp, static_cast<float>(to_u8(c[1])) / fspp,
                            static_cast<float>(to_u8(c[2])) / fspp});
        } else if (KIND == 0) {
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

// 8-B records in full 16-sample slots (the headline's case), without the LDS tile: each
// thread loads its own slot (128 B, eight 16-B loads; the wave's loads cover 64 consecutive
// slots, 8 KB) into registers, the next block's slot while this one is summed. Beside the
// next frame's trace this kernel runs one wave per SIMD: the tile's 64 LDS writes and reads
// per thread and block, and its two barriers per block, were what it waited on there.
// Same sums in the same order as sum_kernel<2, 0> (FR_SUM_DIRECT=0 selects that one).
#ifndef FR_SUM_DIRECT
#define FR_SUM_DIRECT 1
#endif
__global__ __launch_bounds__(kSumThreads) FR_SUM_VGPR_CAP void sum_nib_kernel(
    KParams kp, const float* __restrict__ samples, float* __restrict__ running, float* __restrict__ out_mean,
    uint8_t* __restrict__ out_u8, int first, int last, const float4* __restrict__ att, uint32_t n_prims) {
  __shared__ float4 att16[16];  // level k's entry at byte 16 x nibble (15: the unit entry)
  const uint32_t t = threadIdx.x;
  if (t < 16u) {
    const float4 a = t < n_prims ? att[t] : make_float4(1.0f, 1.0f, 1.0f, 0.0f);
    att16[t] = make_float4(a.x, a.y, a.z, 0.0f);
  }
  const uint32_t q0 = blockIdx.x * kSumThreads, q = q0 + t;
  const uint32_t nq = min(kSumThreads, kp.P - q0);
  uint32_t x = 0, y = 0;
  const bool valid = q < kp.P && slot_xy(kp, q, x, y);
  V3 sum = (first || !valid) ? V3{0.0f, 0.0f, 0.0f} : V3{running[3 * q], running[3 * q + 1], running[3 * q + 2]};
  asm volatile("" : "+v"(sum.x), "+v"(sum.y), "+v"(sum.z));
  __syncthreads();
  typedef float v4f __attribute__((ext_vector_type(4)));
  constexpr uint32_t kV = 2u * kBlockSamples / 4u;  // float4 per slot
  // block bl's slots of this workgroup: one buffer resource (64-bit base, range = its slots),
  // this thread's slot at a 32-bit lane offset; past the last slot the loads return 0
  auto load = [&](uint32_t bl, v4f* v) {
    const float* base = samples + 2u * (static_cast<size_t>(bl * kp.P + q0) * kBlockSamples);
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(base), 0, static_cast<int>(nq * kV * 16u), 0x00020000);
#pragma unroll
    for (uint32_t k = 0; k < kV; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(r, t * (kV * 16u) + k * 16u, 0, 0);
  };
  auto add_block = [&](uint32_t bl, const v4f* v) {
    const uint32_t n = min(kBlockSamples, kp.spp - (kp.b0 + bl) * kBlockSamples);
#pragma unroll
    for (uint32_t j = 0; j < kBlockSamples; ++j) {
      if (j < n) {
        const float tf = (j & 1u) ? v[j >> 1].z : v[j >> 1].x;
        const uint32_t w = __float_as_uint((j & 1u) ? v[j >> 1].w : v[j >> 1].y);
        // the eight entries read before the first multiply: one wave per SIMD runs this
        // beside the trace, and the reads' latency is then not hidden by other waves
        const uint32_t w4 = w << 4;
        float4 e[8];
#pragma unroll
        for (int k = 7; k >= 0; --k) {
          const uint32_t off = (((k & 1) ? w : w4) >> (8 * (k >> 1))) & 0xF0u;
          e[k] = *reinterpret_cast<const float4*>(reinterpret_cast<const char*>(att16) + off);
        }
        V3 col = __float_as_uint(tf) == kDeferAbsorbed ? V3{0.0f, 0.0f, 0.0f} : sky_from_t(tf);
#pragma unroll
        for (int k = 7; k >= 0; --k) col = mul(V3{e[k].x, e[k].y, e[k].z}, col);
        sum = add(sum, col);
      }
    }
  };
  v4f va[kV], vb[kV];
  if (kp.nb) load(0, va);
  for (uint32_t bl = 0; bl < kp.nb; bl += 2u) {
    if (bl + 1u < kp.nb) load(bl + 1u, vb);
    if (valid) add_block(bl, va);
    if (bl + 1u >= kp.nb) break;
    if (bl + 2u < kp.nb) load(bl + 2u, va);
    if (valid) add_block(bl + 1u, vb);
  }
  if (!valid) return;
  if (!last) {
    running[3 * q] = sum.x;
    running[3 * q + 1] = sum.y;
    running[3 * q + 2] = sum.z;
    return;
  }
  const size_t idx = (static_cast<size_t>(y) * kp.W + x) * 3u;
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

hipError_t launch_sum(uint32_t wps, int kind, uint32_t blocks, hipStream_t stream, const KParams& kp,
                      const float* samples, float* running, float* out_mean, uint8_t* out_u8, int first, int last,
                      const float4* att, uint32_t n_prims) {
  const dim3 grid(blocks), block(kSumThreads);
  if (wps == 2 && FR_SUM_DIRECT && kp.ks == kBlockSamples && !(kp.flags & FR_FLAG_MT_BANDS))
    hipLaunchKernelGGL(sum_nib_kernel, grid, block, 0, stream, kp, samples, running, out_mean, out_u8, first, last,
                       att, n_prims);
  else if (wps == 2)
    hipLaunchKernelGGL((sum_kernel<2, 0>), grid, block, 0, stream, kp, samples, running, out_mean, out_u8, first,
                       last, att, n_prims);
  else if (kind == 1)
    hipLaunchKernelGGL((sum_kernel<3, 1>), grid, block, 0, stream, kp, samples, running, out_mean, out_u8, first,
                       last, att, n_prims);
  else
    hipLaunchKernelGGL((sum_kernel<3, 0>), grid, block, 0, stream, kp, samples, running, out_mean, out_u8, first,
                       last, att, n_prims);
  return hipGetLastError();
}

}  // namespace fr
