// pk_rate.hip — issue rate of packed vs plain f32 VALU ops on gfx950 (a microbenchmark for
// profiles/AB_LOG.md): every wave runs N iterations of 16 independent instructions of one
// kind; the kernel's time gives wave-instructions per SIMD-cycle.
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int KIND>
__global__ __launch_bounds__(256) void rate(float* out, int iters) {
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
        a7 = a0 + 7, b0 = a0 + 8, b1 = a0 + 9, b2 = a0 + 10, b3 = a0 + 11, b4 = a0 + 12, b5 = a0 + 13, b6 = a0 + 14,
        b7 = a0 + 15;
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 p0 = {a0, b0}, p1 = {a1, b1}, p2 = {a2, b2}, p3 = {a3, b3}, p4 = {a4, b4}, p5 = {a5, b5}, p6 = {a6, b6},
     p7 = {a7, b7};
  const float m = 0.999f;
  const f2 mm = {m, m};
  for (int i = 0; i < iters; ++i) {
    if constexpr (KIND == 0) {  // 16 plain v_mul_f32
#define M(x) asm volatile("v_mul_f32 %0, %0, %1" : "+v"(x) : "v"(m));
      M(a0) M(a1) M(a2) M(a3) M(a4) M(a5) M(a6) M(a7) M(b0) M(b1) M(b2) M(b3) M(b4) M(b5) M(b6) M(b7)
    } else if constexpr (KIND == 1) {  // 16 v_pk_mul_f32 (32 multiplies)
#define P(x) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(x) : "v"(mm));
      P(p0) P(p1) P(p2) P(p3) P(p4) P(p5) P(p6) P(p7) P(p0) P(p1) P(p2) P(p3) P(p4) P(p5) P(p6) P(p7)
    } else if constexpr (KIND == 2) {  // 16 v_pk_add_f32
#define Q(x) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(x) : "v"(mm));
      Q(p0) Q(p1) Q(p2) Q(p3) Q(p4) Q(p5) Q(p6) Q(p7) Q(p0) Q(p1) Q(p2) Q(p3) Q(p4) Q(p5) Q(p6) Q(p7)
    } else if constexpr (KIND == 3) {  // 16 v_fma_f32
#define F(x) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(m));
      F(a0) F(a1) F(a2) F(a3) F(a4) F(a5) F(a6) F(a7) F(b0) F(b1) F(b2) F(b3) F(b4) F(b5) F(b6) F(b7)
    } else if constexpr (KIND == 4) {  // 16 v_xor_b32
#define X(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(m));
      X(a0) X(a1) X(a2) X(a3) X(a4) X(a5) X(a6) X(a7) X(b0) X(b1) X(b2) X(b3) X(b4) X(b5) X(b6) X(b7)
    } else if constexpr (KIND == 6) {  // 16 v_mul_f32 with an SGPR operand
#define MS(x) asm volatile("v_mul_f32 %0, %1, %0" : "+v"(x) : "s"(m));
      MS(a0) MS(a1) MS(a2) MS(a3) MS(a4) MS(a5) MS(a6) MS(a7) MS(b0) MS(b1) MS(b2) MS(b3) MS(b4) MS(b5) MS(b6) MS(b7)
    } else if constexpr (KIND == 7) {  // 16 v_pk_mul_f32 with an SGPR-pair operand
#define PS(x) asm volatile("v_pk_mul_f32 %0, %1, %0" : "+v"(x) : "s"(mm));
      PS(p0) PS(p1) PS(p2) PS(p3) PS(p4) PS(p5) PS(p6) PS(p7) PS(p0) PS(p1) PS(p2) PS(p3) PS(p4) PS(p5) PS(p6) PS(p7)
    } else if constexpr (KIND == 8) {  // 16 v_add_f32 with an SGPR operand
#define AS(x) asm volatile("v_add_f32 %0, %1, %0" : "+v"(x) : "s"(m));
      AS(a0) AS(a1) AS(a2) AS(a3) AS(a4) AS(a5) AS(a6) AS(a7) AS(b0) AS(b1) AS(b2) AS(b3) AS(b4) AS(b5) AS(b6) AS(b7)
    } else if constexpr (KIND == 9) {  // 16 v_mov_b32
#define MV(x) asm volatile("v_mov_b32 %0, %0" : "+v"(x));
      MV(a0) MV(a1) MV(a2) MV(a3) MV(a4) MV(a5) MV(a6) MV(a7) MV(b0) MV(b1) MV(b2) MV(b3) MV(b4) MV(b5) MV(b6) MV(b7)
    } else if constexpr (KIND == 5) {  // 16 v_max3_f32
#define X3(x, y) asm volatile("v_max3_f32 %0, %0, %1, %1" : "+v"(x) : "v"(y));
      X3(a0, m) X3(a1, m) X3(a2, m) X3(a3, m) X3(a4, m) X3(a5, m) X3(a6, m) X3(a7, m) X3(b0, m) X3(b1, m) X3(b2, m)
      X3(b3, m) X3(b4, m) X3(b5, m) X3(b6, m) X3(b7, m)
    }
  }
  const float s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + b0 + b1 + b2 + b3 + b4 + b5 + b6 + b7 + p0.x + p1.x + p2.x +
                  p3.x + p4.x + p5.x + p6.x + p7.x + p0.y + p1.y + p2.y + p3.y + p4.y + p5.y + p6.y + p7.y;
  if (s == 12345.678f) out[0] = s;
}

int main() {
  float* d;
  hipMalloc(&d, 4);
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  const double ghz = prop.clockRate / 1e6;
  const char* names[] = {"v_mul_f32", "v_pk_mul_f32", "v_pk_add_f32", "v_fma_f32", "v_xor_b32", "v_max3_f32",
                         "v_mul_f32 (sgpr)", "v_pk_mul_f32 (sgpr pair)", "v_add_f32 (sgpr)", "v_mov_b32"};
  const int iters = 20000;
  for (int waves_per_simd = 4; waves_per_simd <= 8; waves_per_simd *= 2) {
    const int blocks = cus * waves_per_simd;  // 256 threads = 4 waves = one per SIMD
    for (int k = 0; k < 10; ++k) {
      hipEvent_t e0, e1;
      hipEventCreate(&e0);
      hipEventCreate(&e1);
      auto launch = [&]() {
        switch (k) {
          case 0: hipLaunchKernelGGL(rate<0>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          case 1: hipLaunchKernelGGL(rate<1>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          case 2: hipLaunchKernelGGL(rate<2>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          case 3: hipLaunchKernelGGL(rate<3>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          case 4: hipLaunchKernelGGL(rate<4>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          case 5: hipLaunchKernelGGL(rate<5>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          case 6: hipLaunchKernelGGL(rate<6>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          case 7: hipLaunchKernelGGL(rate<7>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          case 8: hipLaunchKernelGGL(rate<8>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
          case 9: hipLaunchKernelGGL(rate<9>, dim3(blocks), dim3(256), 0, 0, d, iters); break;
        }
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      const double insts = double(blocks) * 4 * iters * 16;  // wave-instructions
      const double simd_cycles = ms * 1e-3 * ghz * 1e9 * cus * 4;
      printf("{\"inst\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.3f, \"cycles_per_wave_inst\": %.3f, \"clock_ghz\": %.2f}\n",
             names[k], waves_per_simd, ms, simd_cycles / insts, ghz);
    }
  }
  return 0;
}
