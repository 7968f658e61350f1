// sum.h — the launch of sum_kernel (csrc/sum.hip): the per-pixel, in-sample-order sum
// of a pass's sample records (tracer.rs:170-184), and its workgroup size.
//
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "trace_kernel.h"

namespace fr {

#ifndef FR_SUM_THREADS
#define FR_SUM_THREADS 256  // 64 (A/B): one-wave workgroups, no barrier between the slot's waves
#endif
constexpr uint32_t kSumThreads = FR_SUM_THREADS;

// kind: 0 by KParams flags; 1 FR_SKY_DEFER's 12-B records. wps: words per sample record
// (2 or 3).
hipError_t launch_sum(uint32_t wps, int kind, uint32_t blocks, hipStream_t stream, const KParams& kp,
                      const float* samples, float* running, float* out_mean, uint8_t* out_u8, int first, int last,
                      const float4* att, uint32_t n_prims);

}  // namespace fr
