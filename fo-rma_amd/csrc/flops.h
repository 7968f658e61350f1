// flops.h — frozen f32 operation counts of the traced path, for the VALU roofline.
//
// One flop = one f32 add, sub, mul, div, sqrt, min or max of the reference algorithm as
// this build evaluates it (rt_core.h / render.hip); compares, selects, conversions and
// the integer RNG work are not counted. Each constant is counted from the code named
// beside it. bench.py reads this file (every `constexpr double kFlop...` line) and
// forms, per frame of an in-order-loop scene (no BVH):
//
//   flops = segments x (kFlopSegment + sum over primitives of kFlopTest<kind>)
//         + hits x kFlopHit<winner kind> + scatters x (kFlopScatter<class> + kFlopUnwind)
//         + (segments - hits) x kFlopSky + samples x (kFlopCamera + kFlopSum)
//         + pixels x kFlopPixel
//
// from the kernel's exact counters (fr_stats segments / hits / scatters / samples). The
// rejection loops enter at their expected trip counts (1 / acceptance): 4/pi tries per
// lens sample, 6/pi per unit-sphere sample.
#pragma once

namespace fr {

// per segment: 1/d per axis (recip_nr, render.hip closest-hit setup)
constexpr double kFlopSegment = 3;
// ... plus o * inv per axis when the scene has axis-aligned boxes (their slab distances are
// fma(lo, inv, -(o inv)), rt_core.h slab3_box; an fma counts as two flops)
constexpr double kFlopSegmentBox = 3;
// ... plus a = dot(d, d) when the scene has spheres (sphere_root's loop-invariant a)
constexpr double kFlopSegmentSphere = 5;

// closest-hit tests, per primitive per segment
// box, slab3_box + slab_root: fma(lo, inv, -(o inv)), fma(hi, inv, -(o inv)) per axis (12),
// per-axis min and max (6), tn = max of 3 (2), tf = min of 3 (2)
constexpr double kFlopTestBox = 22;
// sphere_root (sphere.rs:23-51): oc (3), b = dot (5), c = dot - r*r (7), disc (3); on
// disc > 0 also sqrt, -b -+ sq, two divides (5): counted as the miss path
constexpr double kFlopTestSphere = 18;
// plane_test (plane.rs:24-44): denom = dot (5); on a pass t (9), p (6), bounds (6):
// counted as the gate only
constexpr double kFlopTestPlane = 5;
// tri_root: two crosses (18), four dots (20), 1/det (1), s (3), three scalings (3), u+v (1)
constexpr double kFlopTestTriangle = 46;
// oriented box: obb_frame (oc 3, two sets of three dots 30, inverse 3) + slab 22
constexpr double kFlopTestObb = 58;

// the winner's record, per hit: p = o + t d (6) plus its normal
constexpr double kFlopHitBox = 6 + 22;     // slab_normal recomputes the winner's slab
constexpr double kFlopHitSphere = 6 + 6;   // (p - c) / r
constexpr double kFlopHitPlane = 6 + 3;    // -orientation
constexpr double kFlopHitTriangle = 6 + 0; // precomputed winding normal
constexpr double kFlopHitObb = 6 + 36 + 22;

// scatter, per successful scatter (sphere.rs:84-152, plane.rs:101-122)
// a unit-sphere rejection try: 3 x (k * 2^-24, 2r - 1) (9) + dot(p, p) (5)
constexpr double kFlopSphereTry = 14;
constexpr double kSphereTries = 1.9098593171027440;  // 6 / pi
// lambertian: (p + n) + r (6), target - p (3)
constexpr double kFlopScatterLambert = 9 + kFlopSphereTry * kSphereTries;
// metal: unit(d) (9), reflect (12), + fuzz * r (6), dot(dir, n) > 0 (5)
constexpr double kFlopScatterMetal = 32 + kFlopSphereTry * kSphereTries;
// dielectric: reflect (12), dot (5), cosine (13), unit (9), dt (5), disc (5), refract (16),
// schlick (11), one draw (1)
constexpr double kFlopScatterDielectric = 77;
// the attenuation product of the unwind, per scatter level
constexpr double kFlopUnwind = 3;

// sky, per missed segment (tracer.rs:211-218): unit (9), t (2), blend (7)
constexpr double kFlopSky = 21;

// per sample: jitter (6), lens tries (2 coordinates x 3 + dot 5 = 11, 4/pi of them), the
// ray (rd 3, offset 9, origin 3, direction 18) (camera.rs:62-72)
constexpr double kFlopCamera = 6 + 11 * 1.2732395447351628 + 3 + 9 + 3 + 18;
// per sample: col = col + c (tracer.rs:174)
constexpr double kFlopSum = 3;
// per pixel: / spp (3), sqrt and * 255 for u8 (6) (tracer.rs:177-184)
constexpr double kFlopPixel = 9;

}  // namespace fr
