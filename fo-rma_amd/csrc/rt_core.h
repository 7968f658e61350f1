// rt_core.h — f32 arithmetic of fo-rma's tracer hot path, shared by the gfx950
// kernel and the host-side camera setup of libforma_rt.
//
// Every expression keeps the reference's IEEE-f32 operation order, because path
// tracing is chaotic: one ulp in a hit distance or a rejection test changes the
// whole path. Build rules (enforced in the Makefile): -ffp-contract=off, no
// fast-math, correctly rounded '/' and sqrt on the device, no denormal flush.
//
// Reference mapping (paths relative to the reference root):
//   V3 ops ............ cpu_ray_tracer/primitives.rs:50-150 (dot :58-60, cross :62-68,
//                       unit_vector :70-72)
//   reflect/refract/schlick ... cpu_ray_tracer/utility.rs:27-54
//   random_in_unit_{circle,sphere} ... utility.rs:4-25 (rejection loops)
//   Rng ............... replaces rand::thread_rng() (rand 0.9.2, Cargo.lock:2735) with a
//                       counter-keyed xoshiro128+ stream per (seed, pixel, 16-sample block)
//   sphere_root ....... shapes/sphere.rs:23-51
//   plane_test ........ shapes/plane.rs:24-44 (stale-record quirk kept)
//   slab3/slab_root ... build-defined box, shaped like Sphere::hit
//   scatter_* ......... shapes/sphere.rs:84-152, shapes/plane.rs:101-122
//   sky ............... cpu_ray_tracer/tracer.rs:211-218
#pragma once
#include <stdint.h>

#if defined(__HIPCC_RTC__)
#define FR_HD __host__ __device__ __forceinline__  // hiprtc (trace_kernel.h's run-time build)
#elif defined(__HIPCC__) || defined(__HIP__)
#include <hip/hip_runtime.h>
#define FR_HD __host__ __device__ __forceinline__
#else
#include <math.h>
#define FR_HD static inline
#endif

namespace fr {

struct V3 {
  float x, y, z;
};

FR_HD V3 mk(float x, float y, float z) { return V3{x, y, z}; }
FR_HD V3 add(V3 a, V3 b) { return V3{a.x + b.x, a.y + b.y, a.z + b.z}; }
FR_HD V3 sub(V3 a, V3 b) { return V3{a.x - b.x, a.y - b.y, a.z - b.z}; }
FR_HD V3 mul(V3 a, V3 b) { return V3{a.x * b.x, a.y * b.y, a.z * b.z}; }
// f32 * Vec3 (primitives.rs:128-138) and Vec3 * f32 (:116-126) are the same products.
FR_HD V3 scl(float s, V3 a) { return V3{s * a.x, s * a.y, s * a.z}; }
FR_HD V3 divs(V3 a, float s) { return V3{a.x / s, a.y / s, a.z / s}; }
// primitives.rs:58-60 — left to right, no fused multiply-add
FR_HD float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
FR_HD V3 cross(V3 a, V3 b) {
  return V3{a.y * b.z - a.z * b.y, -(a.x * b.z - a.z * b.x), a.x * b.y - a.y * b.x};
}
FR_HD float length(V3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
FR_HD V3 unit(V3 a) { return divs(a, length(a)); }  // 3 divides, no reciprocal

// utility.rs:27-30: v - 2*dot(v,n)*n, evaluated as v - ((2*dot) * n)
FR_HD V3 reflect(V3 v, V3 n) { return sub(v, scl(2.0f * dot(v, n), n)); }

// utility.rs:49-54; powi(x,5) is lowered by LLVM's ExpandPowI (and compiler-rt's
// __powisf2) to x * ((x*x)*(x*x)); frozen here.
FR_HD float schlick(float cosine, float ref_idx) {
  float r0 = (1.0f - ref_idx) / (1.0f + ref_idx);
  r0 = r0 * r0;
  float x = 1.0f - cosine;
  float x2 = x * x;
  float x4 = x2 * x2;
  return r0 + (1.0f - r0) * (x * x4);
}

// ---------------------------------------------------------------------------
// RNG. One stream per (seed, pixel, key): key b for block b of 16 samples, and, when
// spp > 16, 2^31 | s / 4 for the 4-sample sub-blocks of the pixel's last block
// (render.hip stream_key). splitmix64 keys a xoshiro128+ 1.0 state (Blackman & Vigna's
// generator for floating-point output: only the upper bits are used); a stream's
// samples draw from it in sample order (the reference's save_image draws every sample
// from one sequential stream, tracer.rs:164-175). f32 = ((u32 ^ 2^31) >> 8) * 2^-24.
// ---------------------------------------------------------------------------
struct Rng {
  uint32_t s0, s1, s2, s3;
};

FR_HD uint64_t splitmix64_next(uint64_t& x) {
  x += 0x9E3779B97F4A7C15ull;
  uint64_t z = x;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

FR_HD Rng rng_seed(uint64_t seed, uint32_t pixel, uint32_t block) {
  uint64_t x = seed ^ ((static_cast<uint64_t>(pixel) << 32) | static_cast<uint64_t>(block));
  uint64_t a = splitmix64_next(x);
  uint64_t b = splitmix64_next(x);
  return Rng{static_cast<uint32_t>(a), static_cast<uint32_t>(a >> 32), static_cast<uint32_t>(b),
             static_cast<uint32_t>(b >> 32)};
}

FR_HD uint32_t rotl32(uint32_t x, int k) { return (x << k) | (x >> (32 - k)); }

FR_HD uint32_t rng_next(Rng& r) {  // xoshiro128+ 1.0
  const uint32_t result = r.s0 + r.s3;
  const uint32_t t = r.s1 << 9;
#if defined(__HIP_DEVICE_COMPILE__) && !defined(FR_XOSHIRO_PLAIN)
  // the same state transition with gfx950's three-input v_bitop3_b32 (0x96 = a ^ b ^ c):
  // s2' = s2 ^ s0 ^ t, s1' = s1 ^ (s2 ^ s0), s0' = s0 ^ (s3 ^ s1), s3' = rotl(s3 ^ s1, 11);
  // 6 VALU per draw instead of 7 (LLVM does not form bitop3 from xor chains); C3 trace
  // 18.50 -> 18.15 ms, bit-identical (FR_XOSHIRO_PLAIN keeps the plain sequence for A/B)
  const uint32_t s3x = r.s3 ^ r.s1;
  const uint32_t s1n = __builtin_amdgcn_bitop3_b32(r.s1, r.s2, r.s0, 0x96);
  const uint32_t s2n = __builtin_amdgcn_bitop3_b32(r.s2, r.s0, t, 0x96);
  r.s0 ^= s3x;
  r.s1 = s1n;
  r.s2 = s2n;
  r.s3 = rotl32(s3x, 11);
#else
  r.s2 ^= r.s0;
  r.s3 ^= r.s1;
  r.s1 ^= r.s2;
  r.s0 ^= r.s3;
  r.s2 ^= t;
  r.s3 = rotl32(r.s3, 11);
#endif
  return result;
}

// f32 in [0, 1): k = (u ^ 2^31) >> 8, r = k * 2^-24 (exact)
FR_HD float rng_f32(Rng& r) {
  return static_cast<float>((rng_next(r) ^ 0x80000000u) >> 8) * 5.9604644775390625e-08f;
}
// 2^24 rng_f32(r): the integer before the scale, as an f32 (exact)
FR_HD float rng_f32_scaled(Rng& r) { return static_cast<float>((rng_next(r) ^ 0x80000000u) >> 8); }

// 2*r - 1 for that r: (k - 2^23) * 2^-23 is exact in f32 and equals the arithmetic
// shift (int32)u >> 8 scaled by 2^-23, so shift + convert + scale replace the
// reference's 2*r - 1 bit for bit.
FR_HD float rng_signed_unit(Rng& r) {
  return static_cast<float>(static_cast<int32_t>(rng_next(r)) >> 8) * 1.1920928955078125e-07f;
}

// The same value scaled by 2^23: the integer (int32)u >> 8 as an f32 (exact). A
// rejection test on these, dot(k, k) >= 2^46, takes the same decision as dot(p, p) >= 1
// on p = k * 2^-23: every product and sum is the unscaled one times 2^46 exactly (f32
// rounding commutes with power-of-two scaling away from the denormal and overflow
// ranges, and 1 <= k*k <= 2^46 or k = 0). The accepted point is scaled once.
FR_HD float rng_signed_unit_scaled(Rng& r) { return static_cast<float>(static_cast<int32_t>(rng_next(r)) >> 8); }
constexpr float kSignedUnitScale = 1.1920928955078125e-07f;  // 2^-23
constexpr float kUnitBallScaled = 70368744177664.0f;         // 2^46

// utility.rs:4-13: p = 2*(r1, r2, 0) - (1, 1, 0), retry while dot(p,p) >= 1
#ifndef FR_LENS_TRY
#define FR_LENS_TRY()
#define FR_RUS_TRY()
#endif
FR_HD V3 random_in_unit_circle(Rng& r) {
  float px, py;
  do {
    FR_LENS_TRY();
    px = rng_signed_unit(r);
    py = rng_signed_unit(r);
    // dot(p,p) = (px*px + py*py) + 0*0; adding +0 to a sum of squares is exact
  } while (px * px + py * py >= 1.0f);
  return V3{px, py, 0.0f};
}

// utility.rs:15-25: p = 2*(r1, r2, r3) - (1, 1, 1), retry while dot(p,p) >= 1
FR_HD V3 random_in_unit_sphere(Rng& r) {
  float px, py, pz;
  do {
    FR_RUS_TRY();
    px = rng_signed_unit(r);
    py = rng_signed_unit(r);
    pz = rng_signed_unit(r);
  } while (px * px + py * py + pz * pz >= 1.0f);
  return V3{px, py, pz};
}

// ---------------------------------------------------------------------------
// Primitives. The closest-hit loop (tracer.rs:190-200) only needs each test's
// accepted t; the hit record's point and normal are formed once for the winner
// (DESIGN.md §4.2 shows this equals the reference's shared-record updates).
// ---------------------------------------------------------------------------

// shapes/sphere.rs:23-51 without the record writes; a = dot(d, d) (loop-invariant).
// Both roots are formed unconditionally (no side effects) and the near one wins.
// rr = RN(radius * radius), the product the test forms (the BVH's leaf records carry it in
// place of the radius, render.hip)
FR_HD bool sphere_root_rr(V3 c, float rr, V3 o, V3 d, float a, float t_min, float t_max, float& t) {
  const V3 oc = sub(o, c);
  const float b = dot(oc, d);
  const float cc = dot(oc, oc) - rr;
  const float disc = b * b - a * cc;
  if (disc > 0.0f) {
    const float sq = sqrtf(disc);
    const float r1 = (-b - sq) / a;
    const float r2 = (-b + sq) / a;
    const bool c1 = r1 > t_min && r1 < t_max;
    const bool c2 = r2 > t_min && r2 < t_max;
    t = c1 ? r1 : r2;
    return c1 || c2;
  }
  return false;
}
FR_HD bool sphere_root(V3 c, float radius, V3 o, V3 d, float a, float t_min, float t_max, float& t) {
  return sphere_root_rr(c, radius * radius, o, d, a, t_min, t_max, t);
}

// shapes/plane.rs:24-44. denom is compared against the t-range; when it passes,
// the record's t (and p = point_at(t)) are written before the bounds test, so a
// failed test leaves them stale (returns 1); t may be negative. Returns 2 on a hit.
FR_HD int plane_test(V3 pos, V3 orient, V3 size, V3 o, V3 d, float t_min, float t_max, float& t) {
  const float denom = dot(orient, d);
  if (denom > t_min && denom < t_max) {
    t = dot(sub(pos, o), orient) / denom;
    const V3 p = add(o, scl(t, d));
    const bool in = p.x > pos.x - size.x && p.x < pos.x + size.x && p.y > pos.y - size.y &&
                    p.y < pos.y + size.y && p.z > pos.z - size.z && p.z < pos.z + size.z;
    return in ? 2 : 1;
  }
  return 0;
}

// Build-defined box. Per axis k, with inv_k = 1/d_k:
//   t0_k = (lo_k - o_k) * inv_k,  t1_k = (hi_k - o_k) * inv_k
//   near_k = minNum(t0_k, t1_k),  far_k = maxNum(t0_k, t1_k)   (IEEE 754-2008, NaN-ignoring)
//   tn = maxNum(maxNum(near_x, near_y), near_z),  tf = minNum(minNum(far_x, far_y), far_z)
// Hit iff tn < tf and one root lies in (t_min, t_max); the near root wins (Sphere::hit's
// two-root shape). The normal is the outward face normal of the first axis (x, y, z order)
// whose near (far) value equals tn (tf): -sign(d_k) on entry, +sign(d_k) on exit,
// with sign(0) counted negative. Zero signs never matter (t is only compared, never 0
// when accepted), so the hardware min/max agree with the host's fminf/fmaxf.
// v_min_f32 / v_max_f32 / v_min3_f32 directly: the generic lowering of fminf/fmaxf
// re-canonicalises operands it cannot prove canonical (every result of an asm statement),
// one v_max_f32 x, x, x per shared slab value in the scene kernel's list walk
FR_HD float fmin_num(float a, float b) {
#if defined(__HIP_DEVICE_COMPILE__)
  float r;
  asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  return fminf(a, b);
#endif
}
FR_HD float fmax_num(float a, float b) {
#if defined(__HIP_DEVICE_COMPILE__)
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
#else
  return fmaxf(a, b);
#endif
}
// minNum(minNum(a, b), c) in one v_min3_f32 (device-checked against the chained v_min_f32
// and the host's fminf chain: test_device_max3_and_min3_match_fmaxf_fminf)
FR_HD float fmin3_num(float a, float b, float c) {
#if defined(__HIP_DEVICE_COMPILE__)
  float r;
  asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
#else
  return fminf(fminf(a, b), c);
#endif
}

#if defined(__HIP__)
// v_rcp_f32 (1 ulp) refined by one FMA Newton step: r' = r + r (1 - x r). Equal to the
// correctly rounded 1.0f / x for every x whose exponent field is in [kRecipExpLo,
// kRecipExpHi] (exhaustively checked on the device: fr_selftest_recip,
// tests/test_gpu_parity.py::test_recip_nr_exhaustive); callers take 1.0f / x elsewhere.
__device__ __forceinline__ float recip_nr(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const float r = __builtin_amdgcn_rcpf(x);
  const float e = __builtin_fmaf(-x, r, 1.0f);
  return __builtin_fmaf(e, r, r);
#else
  return 1.0f / x;  // not used on the host
#endif
}

// Reciprocal as the parity contract needs it (correctly rounded): recip_nr inside its
// exhaustively checked range, the full IEEE division otherwise (zero, denormals,
// |x| >= 2^126, inf, NaN). The fallback is a real branch, skipped by waves with no such lane.
__device__ __forceinline__ bool recip_nr_ok(float x) {
  const float ax = __builtin_fabsf(x);
  return (ax >= 0x1p-126f) & (ax < 0x1p126f);
}

// a / b correctly rounded, given y = RN(1 / b): q0 = a y and one FMA residual correction
// q0 + (a - b q0) y (Markstein's step; the compiler's IEEE sequence takes two, as its y is
// v_rcp_f32's 1-ulp estimate). Its v_div_scale / v_div_fmas / v_div_fixup steps are
// identities when a = +0 or |a| in [2^-100, 2^100] and |b| in [2^-100, 2^100] (no operand,
// quotient or residual near the denormal / overflow range), and there every operand pair
// scales to one in [1, 2) x [1, 2) by powers of two that scale both results exactly: all
// 2^46 such pairs are checked on the device (fr_selftest_div,
// tests/test_gpu_parity.py::test_div_rn_exhaustive). Used only where the operand ranges
// hold by construction. FR_DIV_2STEP: the second correction as well (the round-4 form).
__device__ __forceinline__ float div_rn(float a, float b, float y) {
  const float q0 = a * y;
  const float q1 = __builtin_fmaf(__builtin_fmaf(-b, q0, a), y, q0);
#ifdef FR_DIV_2STEP
  return __builtin_fmaf(__builtin_fmaf(-b, q1, a), y, q1);
#else
  return q1;
#endif
}
#endif

#if defined(__HIP__)
// Correctly rounded sqrt(x) for x in [2^-96, 2^126]: v_sqrt_f32 and the compiler's two
// FMA residual corrections, without its denormal scaling and class fix-up (identities in
// that range; the same core as sky_t_fast, fr_selftest_ops op 14).
__device__ __forceinline__ float sqrt_core(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sdn = __uint_as_float(__float_as_uint(s) - 1u);
  const float sup = __uint_as_float(__float_as_uint(s) + 1u);
  const float rdn = __builtin_fmaf(-sdn, s, x);
  const float rup = __builtin_fmaf(-sup, s, x);
  float r = rdn <= 0.0f ? sdn : s;
  return rup > 0.0f ? sup : r;
#else
  return sqrtf(x);  // not used on the host
#endif
}

// The segment's part of sphere_root_fast: ya = RN(1 / a) and whether a = dot(d, d) is in
// [2^-60, 2^60] (recip_nr is exact there).
struct SphereSeg {
  float ya;
  bool ok;
};
__device__ __forceinline__ SphereSeg sphere_seg(float a) {
  return SphereSeg{recip_nr(a), (a >= 0x1p-60f) && (a <= 0x1p60f)};
}

// sphere_root bit for bit, with the root's sqrt and its two divisions by a done by their
// core sequences (sqrt_core, div_rn with the segment's ya) on lanes where disc is in
// [2^-96, 2^126], |b| <= 2^40 and a in [2^-60, 2^60]; other lanes take sphere_root's
// expressions. There |-b -+ sq| <= 2^41 and a root that can be accepted (> t_min = 0.001)
// has |numerator| >= 0.001 a >= 2^-70, so the numerator, the quotient (<= 2^101) and
// every intermediate are normal and div_rn is the correctly rounded quotient; a root below
// 0.001 in magnitude is below it by either sequence (a numerator under 2^-70 gives
// |q| < 2^-10 with an absolute error far below the gap), so both reject it. Checked against
// sphere_root on the device by fr_selftest_ops op 16 (tests/test_gpu_parity.py).
// (split in two so that a caller can mark the root step as its own region: the BVH leaf
// test, tools/isa_sections.py)
struct SphereDisc {
  float b, disc;
};
__device__ __forceinline__ SphereDisc sphere_disc_rr(V3 c, float rr, V3 o, V3 d, float a) {
  const V3 oc = sub(o, c);
  const float b = dot(oc, d);
  const float cc = dot(oc, oc) - rr;
  return SphereDisc{b, b * b - a * cc};
}
__device__ __forceinline__ SphereDisc sphere_disc(V3 c, float radius, V3 o, V3 d, float a) {
  return sphere_disc_rr(c, radius * radius, o, d, a);
}
// the roots of a sphere test whose discriminant is > 0
__device__ __forceinline__ bool sphere_roots_fast(SphereDisc q, float a, SphereSeg sg, float t_min, float t_max,
                                                  float& t) {
  const float b = q.b, disc = q.disc;
  {
    float r1, r2;
    const bool fast = static_cast<int>(sg.ok) & static_cast<int>(disc >= 0x1p-96f) & static_cast<int>(disc <= 0x1p126f) &
                      static_cast<int>(__builtin_fabsf(b) <= 0x1p40f);
    if (fast) {
      const float sq = sqrt_core(disc);
      r1 = div_rn(-b - sq, a, sg.ya);
      r2 = div_rn(-b + sq, a, sg.ya);
    } else {
      const float sq = sqrtf(disc);
      r1 = (-b - sq) / a;
      r2 = (-b + sq) / a;
    }
    const bool c1 = r1 > t_min && r1 < t_max;
    const bool c2 = r2 > t_min && r2 < t_max;
    t = c1 ? r1 : r2;
    return c1 || c2;
  }
}
__device__ __forceinline__ bool sphere_root_fast(V3 c, float radius, V3 o, V3 d, float a, SphereSeg sg,
                                                 float t_min, float t_max, float& t) {
  const SphereDisc q = sphere_disc(c, radius, o, d, a);
  if (q.disc > 0.0f) return sphere_roots_fast(q, a, sg, t_min, t_max, t);
  return false;
}
#endif

// maxNum(maxNum(a, b), c) in one v_max3_f32 (same IEEE-mode NaN rule as the chained
// v_max_f32; device-checked against fmaxf chains in test_device_max3_matches_fmaxf).
FR_HD float fmax3_num(float a, float b, float c) {
#if defined(__HIP_DEVICE_COMPILE__)
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
#else
  return fmaxf(fmaxf(a, b), c);
#endif
}

struct Slab {
  V3 t0, t1;  // slab distances per axis
  float tn, tf;
};

FR_HD Slab slab3(V3 lo, V3 hi, V3 o, V3 inv) {
  Slab s;
  // scalar f32 ops: packed v_pk_add/mul_f32 cost more issue time than two plain ops
  // (MI355X_MICROARCH.md, "vector-instruction ISSUE cost"; measured -2% here)
  s.t0 = V3{(lo.x - o.x) * inv.x, (lo.y - o.y) * inv.y, (lo.z - o.z) * inv.z};
  s.t1 = V3{(hi.x - o.x) * inv.x, (hi.y - o.y) * inv.y, (hi.z - o.z) * inv.z};
  s.tn = fmax3_num(fmin_num(s.t0.x, s.t1.x), fmin_num(s.t0.y, s.t1.y), fmin_num(s.t0.z, s.t1.z));
  s.tf = fmin3_num(fmax_num(s.t0.x, s.t1.x), fmax_num(s.t0.y, s.t1.y), fmax_num(s.t0.z, s.t1.z));
  return s;
}

// The same slab distances as fma(lo, inv, -o inv) with oinv = o inv precomputed: not
// the box primitive's exact arithmetic, only for the BVH's padded cull boxes (bvh.h).
// One slab distance fma(c, inv, -oinv). A plane at a compile-time 0 (the scene kernel's
// constants) is -oinv: 0 * inv is a zero for the finite (clamped) inv of the box test and the
// cull, so the two differ at most in the sign of a zero distance, which neither root
// selection (t > t_min) nor the face test (t equal to a distance) can see.
FR_HD float slab_d(float c, float inv, float oinv) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (__builtin_constant_p(c) && c == 0.0f) return -oinv;
#endif
  return fmaf(c, inv, -oinv);
}
FR_HD Slab slab3_fused(V3 lo, V3 hi, V3 oinv, V3 inv) {
  Slab s;
  s.t0 = V3{slab_d(lo.x, inv.x, oinv.x), slab_d(lo.y, inv.y, oinv.y), slab_d(lo.z, inv.z, oinv.z)};
  s.t1 = V3{slab_d(hi.x, inv.x, oinv.x), slab_d(hi.y, inv.y, oinv.y), slab_d(hi.z, inv.z, oinv.z)};
  s.tn = fmax3_num(fmin_num(s.t0.x, s.t1.x), fmin_num(s.t0.y, s.t1.y), fmin_num(s.t0.z, s.t1.z));
  s.tf = fmin3_num(fmax_num(s.t0.x, s.t1.x), fmax_num(s.t0.y, s.t1.y), fmax_num(s.t0.z, s.t1.z));
  return s;
}

// The build-defined box's slab distances: fma(lo, inv, -(o inv))
// with inv = RN(1 / d) clamped to +-2^100, one rounding per distance instead of the two of
// (lo - o) * inv, and one instruction per distinct slab coordinate of the scene kernel (o inv
// is per segment): C3 14.84 -> 14.48 ms per streamed frame (profiles/r06e_ab_boxfma.log).
// The clamp keeps zero and tiny direction components finite (inf * lo - inf * o would be
// NaN). FR_BOX_FMA=0 builds the round-5 form (A/B; the oracle's OR_BOX_FMA=0 matches it).
#ifndef FR_BOX_FMA
#define FR_BOX_FMA 1
#endif
constexpr float kBoxInvClamp = 0x1p100f;
FR_HD float box_inv_clamp(float inv) { return fmin_num(fmax_num(inv, -kBoxInvClamp), kBoxInvClamp); }
// recip_nr's range narrowed to |x| >= 2^-100: there RN(1 / x) is within the clamp
FR_HD bool recip_box_ok(float x) {
  const float ax = __builtin_fabsf(x);
  return (ax >= 0x1p-100f) & (ax < 0x1p126f);
}
FR_HD Slab slab3_box(V3 lo, V3 hi, V3 o, V3 inv, V3 oinv) {
  if (FR_BOX_FMA) return slab3_fused(lo, hi, oinv, inv);
  (void)oinv;
  return slab3(lo, hi, o, inv);
}

// Root selection: returns true and the accepted t if the box is hit in (t_min, t_max).
// Equivalent branch-free form of "near root if tn in (t_min, t_max), else far root if
// tf in (t_min, t_max), and tn < tf": when tn > t_min the far root can only be taken
// if tn >= t_max, and then tf > tn >= t_max fails too.
FR_HD bool slab_root(const Slab& s, float t_min, float t_max, float& t) {
  t = s.tn > t_min ? s.tn : s.tf;
  return (t > t_min) & (t < t_max) & (s.tn < s.tf);
}

FR_HD float comp(V3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }

FR_HD V3 axis_normal(int k, float s) {
  return V3{k == 0 ? s : 0.0f, k == 1 ? s : 0.0f, k == 2 ? s : 0.0f};
}

// Outward normal of the accepted root t (t == tn: entry face, else exit face), in the
// frame whose ray direction is dd.
FR_HD V3 slab_normal(const Slab& s, float t, V3 dd) {
#if defined(__HIP_DEVICE_COMPILE__)
  // Branch-free form of the two cases below, for t == tn or t == tf (slab_root's roots;
  // the caller recomputes the winner's slab with the same operations): entry iff t == tn;
  // the first axis whose near (entry) or far (exit) distance equals t; the sign is
  // -sign(d_k) on entry and +sign(d_k) on exit, sign(0) counted negative. Selects on lane
  // masks instead of a divergent branch in which both cases ran for a mixed wave.
  // (both per-axis extremes formed up front: a conditional asm min/max became a branch)
  const bool entry = t == s.tn;
  const float mnx = fmin_num(s.t0.x, s.t1.x), mxx = fmax_num(s.t0.x, s.t1.x);
  const float mny = fmin_num(s.t0.y, s.t1.y), mxy = fmax_num(s.t0.y, s.t1.y);
  const bool kx = (entry ? mnx : mxx) == t;
  const bool ky = !kx && (entry ? mny : mxy) == t;
  const bool kz = !kx && !ky;
  const float dk = kx ? dd.x : (ky ? dd.y : dd.z);
  const float sg = ((dk > 0.0f) != entry) ? 1.0f : -1.0f;
  return V3{kx ? sg : 0.0f, ky ? sg : 0.0f, kz ? sg : 0.0f};
#else
  if (t == s.tn) {
    const int k = fmin_num(s.t0.x, s.t1.x) == s.tn ? 0 : (fmin_num(s.t0.y, s.t1.y) == s.tn ? 1 : 2);
    return axis_normal(k, comp(dd, k) > 0.0f ? -1.0f : 1.0f);
  }
  const int k = fmax_num(s.t0.x, s.t1.x) == s.tf ? 0 : (fmax_num(s.t0.y, s.t1.y) == s.tf ? 1 : 2);
  return axis_normal(k, comp(dd, k) > 0.0f ? 1.0f : -1.0f);
#endif
}

// Build-defined triangle: Moller-Trumbore in f32 with this order;
// e1 = v1 - v0, e2 = v2 - v0 come precomputed (same host f32 ops as the oracle's).
// NaN or infinite barycentrics (det = 0) fail the comparisons.
FR_HD bool tri_root(V3 v0, V3 e1, V3 e2, V3 o, V3 d, float t_min, float t_max, float& t) {
  const V3 pv = cross(d, e2);
  const float inv_det = 1.0f / dot(e1, pv);
  const V3 s = sub(o, v0);
  const float u = dot(s, pv) * inv_det;
  const V3 qv = cross(s, e1);
  const float v = dot(d, qv) * inv_det;
  t = dot(e2, qv) * inv_det;
  return (u >= 0.0f) & (v >= 0.0f) & (u + v <= 1.0f) & (t > t_min) & (t < t_max);
}

// Oriented box: the same slab test in the box frame (rows ax, ay, az of world->local).
struct ObbFrame {
  V3 dl, inv, ol;
};

FR_HD ObbFrame obb_frame(V3 c, V3 ax, V3 ay, V3 az, V3 o, V3 d) {
  ObbFrame f;
  const V3 oc = sub(o, c);
  f.ol = V3{dot(ax, oc), dot(ay, oc), dot(az, oc)};
  f.dl = V3{dot(ax, d), dot(ay, d), dot(az, d)};
  f.inv = V3{1.0f / f.dl.x, 1.0f / f.dl.y, 1.0f / f.dl.z};
  return f;
}

FR_HD V3 obb_normal(V3 ax, V3 ay, V3 az, const Slab& s, float t, V3 dl) {
  const V3 nl = slab_normal(s, t, dl);  // one component is +-1
  const float sg = nl.x + nl.y + nl.z;
  const V3 axis = nl.x != 0.0f ? ax : (nl.y != 0.0f ? ay : az);
  return scl(sg, axis);
}

// ---------------------------------------------------------------------------
// Scatter. Effective classes after the per-shape fallbacks (sphere.rs:56-69,
// plane.rs:48-59): boxes follow the sphere's material table.
// ---------------------------------------------------------------------------
enum ScatterClass : uint32_t { SC_LAMBERT = 0, SC_METAL = 1, SC_DIELECTRIC = 2, SC_LIGHT = 3, SC_NONE = 4 };

// sphere.rs:84-89 / 147-152, plane.rs:101-106: target = (p + n) + rus; dir = target - p
FR_HD V3 scatter_lambert(V3 p, V3 n, Rng& r) {
  const V3 target = add(add(p, n), random_in_unit_sphere(r));
  return sub(target, p);
}

// sphere.rs:91-105, plane.rs:108-122: rus is drawn even when fuzz = 0
FR_HD bool scatter_metal(V3 d, V3 p_unused, V3 n, float fuzz, Rng& r, V3& dir) {
  (void)p_unused;
  const V3 refl = reflect(unit(d), n);
  dir = add(refl, scl(fuzz, random_in_unit_sphere(r)));
  return dot(dir, n) > 0.0f;
}

// sphere.rs:107-145 (ref_idx 1.3; attenuation = colour, applied by the caller)
FR_HD V3 scatter_dielectric(V3 d, V3 n, Rng& r) {
  const float ref_idx = 1.3f;
  const V3 reflected = reflect(d, n);
  V3 outward;
  float ni, cosine;
  const float dn = dot(d, n);
  if (dn > 0.0f) {
    outward = sub(V3{0.0f, 0.0f, 0.0f}, n);
    ni = ref_idx;
    cosine = ref_idx * dot(d, n) / length(d);
  } else {
    outward = n;
    ni = 1.0f / ref_idx;
    cosine = -dot(d, n) / length(d);
  }
  // utility.rs:37-47
  const V3 uv = unit(d);
  const float dt = dot(uv, outward);
  const float disc = 1.0f - ni * ni * (1.0f - dt * dt);
  V3 refracted = V3{0.0f, 0.0f, 0.0f};
  float reflect_prob;
  if (disc > 0.0f) {
    refracted = sub(scl(ni, sub(uv, scl(dt, outward))), scl(sqrtf(disc), outward));
    reflect_prob = schlick(cosine, ref_idx);
  } else {
    reflect_prob = 1.0f;
  }
  return rng_f32(r) < reflect_prob ? reflected : refracted;
}

// tracer.rs:211-218
// split in two for the deferred unwind (render.hip): the blend parameter t, and the colour
FR_HD float sky_t(V3 d) {
  const V3 ud = unit(d);
  return 0.5f * (ud.y + 1.0f);
}
// sky_t from the two values it depends on, d.y and dot(d, d) in length()'s order: the same
// operations (a division by the correctly rounded sqrt, then the blend parameter)
FR_HD float sky_t_from(float dy, float dd) { return 0.5f * (dy / sqrtf(dd) + 1.0f); }
FR_HD V3 sky_from_t(float t) { return add(scl(1.0f - t, V3{1.0f, 1.0f, 1.0f}), scl(t, V3{0.5f, 0.7f, 1.0f})); }
FR_HD V3 sky(V3 d) { return sky_from_t(sky_t(d)); }

#if defined(__HIP__)
// sky_t (tracer.rs:211-218's blend parameter 0.5 (unit(d).y + 1)) with the correctly
// rounded sqrt and division done by their core sequences where the operands allow it:
// v_sqrt_f32 and the compiler's two FMA residual corrections without the denormal
// scaling and class fix-up (identities for dd in [2^-96, 2^126]); and d.y / len by
// div_rn(d.y, len, recip_nr(len)) (recip_nr exact for len's exponent range there, div_rn's
// steps identities for |d.y| in {0} u [2^-100, 2^63], and |d.y| <= len <= 2^63). A d.y
// below 2^-100 in magnitude needs no guard of its own: with len >= 2^-48 both sequences
// give |q| < 2^-50 (the core one's residual may be denormal there), and 1 + q = 1 either
// way. Other lanes take the plain expression. Bit-identical to sky_t: fr_selftest_ops op 14.
__device__ __forceinline__ float sky_t_fast_from(float dy, float dd) {
  const bool fast = (dd >= 0x1p-96f) & (dd <= 0x1p126f);
  if (fast) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float s = __builtin_amdgcn_sqrtf(dd);
    const float sdn = __uint_as_float(__float_as_uint(s) - 1u);
    const float sup = __uint_as_float(__float_as_uint(s) + 1u);
    const float rdn = __builtin_fmaf(-sdn, s, dd);
    const float rup = __builtin_fmaf(-sup, s, dd);
    float len = rdn <= 0.0f ? sdn : s;
    len = rup > 0.0f ? sup : len;
    const float q = div_rn(dy, len, recip_nr(len));
    return 0.5f * (q + 1.0f);
#endif
  }
  return sky_t_from(dy, dd);  // = sky_t(d): the same operations on the same values
}
__device__ __forceinline__ float sky_t_fast(V3 d) {
  return sky_t_fast_from(d.y, d.x * d.x + d.y * d.y + d.z * d.z);  // length()'s sum, in its order
}
#endif

// tracer.rs:182-184: Rust `as u8` saturates (NaN -> 0) and truncates toward zero.
FR_HD uint8_t to_u8(float c) {
  const float s = sqrtf(c) * 255.0f;
  if (!(s > 0.0f)) return 0;
  if (s >= 255.0f) return 255;
  return static_cast<uint8_t>(s);
}

// Rust `f32 as u8` of a value already in byte units: NaN -> 0, saturating, truncation
FR_HD uint8_t as_u8_trunc(float v) {
  if (!(v > 0.0f)) return 0;
  if (v >= 255.0f) return 255;
  return static_cast<uint8_t>(v);
}

}  // namespace fr
