// oracle.cpp — CPU restatement of fo-rma's per-pixel ray/shade loop.
//
// TEST INFRASTRUCTURE ONLY. This file is the parity oracle: only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only
// as the checker or the timed CPU baseline, never as the product path. It shares
// no code with fo-rma_amd/ (the product): it is written in the reference's own
// shape — a Vec3 with operator overloads, a virtual Hitable per shape, a
// recursive get_color — so that agreement with the GPU kernel is evidence, not
// tautology.
//
// Parity status: pinned by (1) the reference's own Vec3 known-answer tests
// (cpu_ray_tracer/primitives.rs:159-255), (2) analytic KATs in tests/, and
// (3) golden fixtures in tests/golden/ made by this oracle. The reference
// itself cannot be built here (Rust toolchain absent; Cargo.toml:22 needs the
// missing ../kopek) and draws from an OS-seeded ThreadRng (rand 0.9.2,
// Cargo.lock:2735), so end-to-end image parity with the Rust binary is
// unpinnable; the RNG is replaced by a counter-keyed stream.
//
// Build: g++ -O2 -ffp-contract=off -fno-fast-math (see oracle/Makefile).
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <memory>
#include <thread>
#include <vector>

namespace {

// ---- cpu_ray_tracer/primitives.rs:4-157 -----------------------------------
struct Vec3 {
  float x, y, z;
  Vec3() : x(0), y(0), z(0) {}
  Vec3(float a, float b, float c) : x(a), y(b), z(c) {}
  static Vec3 zero() { return Vec3(0.0f, 0.0f, 0.0f); }
  static Vec3 one() { return Vec3(1.0f, 1.0f, 1.0f); }
  float r() const { return x; }
  float g() const { return y; }
  float b() const { return z; }
  float length_squared() const { return x * x + y * y + z * z; }         // :50-52
  float length() const { return sqrtf(length_squared()); }              // :54-56
  static float dot(Vec3 a, Vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }  // :58-60
  static Vec3 cross(Vec3 a, Vec3 b) {                                    // :62-68
    return Vec3(a.y * b.z - a.z * b.y, -(a.x * b.z - a.z * b.x), a.x * b.y - a.y * b.x);
  }
  Vec3 unit_vector() const;                                              // :70-72
  Vec3 sqrt() const { return Vec3(sqrtf(x), sqrtf(y), sqrtf(z)); }       // :74-76
};
inline Vec3 operator+(Vec3 a, Vec3 b) { return Vec3(a.x + b.x, a.y + b.y, a.z + b.z); }  // :80-90
inline Vec3 operator-(Vec3 a, Vec3 b) { return Vec3(a.x - b.x, a.y - b.y, a.z - b.z); }  // :92-102
inline Vec3 operator*(Vec3 a, Vec3 b) { return Vec3(a.x * b.x, a.y * b.y, a.z * b.z); }  // :104-114
inline Vec3 operator*(Vec3 a, float s) { return Vec3(a.x * s, a.y * s, a.z * s); }       // :116-126
inline Vec3 operator*(float s, Vec3 a) { return Vec3(s * a.x, s * a.y, s * a.z); }       // :128-138
inline Vec3 operator/(Vec3 a, float s) { return Vec3(a.x / s, a.y / s, a.z / s); }       // :140-150
Vec3 Vec3::unit_vector() const { return *this / length(); }

// ---- cpu_ray_tracer/ray.rs -------------------------------------------------
struct Ray {
  Vec3 from, to;
  Ray() {}
  Ray(Vec3 a, Vec3 b) : from(a), to(b) {}
  Vec3 origin() const { return from; }
  Vec3 direction() const { return to; }
  Vec3 point_at(float t) const { return from + t * to; }  // :26-28
};
struct HitRecord {
  float t = 0.0f;
  Vec3 p, normal;
};
struct ReflectRecord {
  Ray scattered;
  Vec3 attenuation;
};

// ---- the RNG that replaces rand::thread_rng() -------------------------------
// splitmix64 (Steele, Lea & Flood 2014) keys xoshiro128+ 1.0 (Blackman & Vigna
// 2018) per (seed, pixel, stream key); a pixel's samples draw from their streams in
// order (stream_start below; the reference's save_image draws every sample from one
// sequential ThreadRng, tracer.rs:164-175); f32 = ((u32 ^ 2^31) >> 8) * 2^-24.
struct Rng {
  uint32_t s[4];
  static uint64_t splitmix(uint64_t& x) {
    x += 0x9E3779B97F4A7C15ull;
    uint64_t z = x;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  Rng(uint64_t seed, uint32_t pixel, uint32_t sample) {
    uint64_t x = seed ^ ((uint64_t(pixel) << 32) | uint64_t(sample));
    uint64_t a = splitmix(x), b = splitmix(x);
    s[0] = uint32_t(a);
    s[1] = uint32_t(a >> 32);
    s[2] = uint32_t(b);
    s[3] = uint32_t(b >> 32);
  }
  static uint32_t rotl(uint32_t v, int k) { return (v << k) | (v >> (32 - k)); }
  uint32_t next_u32() {
    uint32_t result = s[0] + s[3];
    uint32_t t = s[1] << 9;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 11);
    return result;
  }
  float gen_f32() { return float((next_u32() ^ 0x80000000u) >> 8) * (1.0f / 16777216.0f); }
};

// Stream layout of one pixel's spp samples: blocks of 16 consecutive samples, block b
// drawing from stream key b; when spp > 16, the last block (the one holding sample
// spp - 1) is split into sub-blocks of 4 samples, the one starting at sample s drawing
// from stream key 2^31 | s / 4. True when sample s starts a stream, with its key.
bool stream_start(uint32_t s, uint32_t spp, uint32_t& key) {
  const uint32_t last_block = (spp - 1) / 16;
  if (spp > 16 && s / 16 == last_block) {
    if (s % 4 != 0) return false;
    key = 0x80000000u | (s / 4);
    return true;
  }
  if (s % 16 != 0) return false;
  key = s / 16;
  return true;
}

// ---- cpu_ray_tracer/utility.rs ---------------------------------------------
Vec3 random_in_unit_circle(Rng& rng) {  // :4-13
  float a = rng.gen_f32();
  float b = rng.gen_f32();
  Vec3 p = 2.0f * Vec3(a, b, 0.0f) - Vec3(1.0f, 1.0f, 0.0f);
  while (Vec3::dot(p, p) >= 1.0f) {
    a = rng.gen_f32();
    b = rng.gen_f32();
    p = 2.0f * Vec3(a, b, 0.0f) - Vec3(1.0f, 1.0f, 0.0f);
  }
  return p;
}

Vec3 random_in_unit_sphere(Rng& rng) {  // :15-25
  float a = rng.gen_f32();
  float b = rng.gen_f32();
  float c = rng.gen_f32();
  Vec3 p = 2.0f * Vec3(a, b, c) - Vec3(1.0f, 1.0f, 1.0f);
  while (Vec3::dot(p, p) >= 1.0f) {
    a = rng.gen_f32();
    b = rng.gen_f32();
    c = rng.gen_f32();
    p = 2.0f * Vec3(a, b, c) - Vec3(1.0f, 1.0f, 1.0f);
  }
  return p;
}

Vec3 reflect(Vec3 v, Vec3 n) { return v - 2.0f * Vec3::dot(v, n) * n; }  // :27-30

bool refract(Vec3 v, Vec3 n, float ni_over_nt, Vec3& refracted) {  // :37-47
  Vec3 uv = v.unit_vector();
  float dt = Vec3::dot(uv, n);
  float discriminant = 1.0f - ni_over_nt * ni_over_nt * (1.0f - dt * dt);
  if (discriminant > 0.0f) {
    refracted = ni_over_nt * (uv - dt * n) - sqrtf(discriminant) * n;
    return true;
  }
  return false;
}

// compiler-rt __powisf2 (what f32::powi lowers to without optimisation; LLVM's
// ExpandPowI produces the same product order with it)
float powi(float a, int b) {
  const bool recip = b < 0;
  float r = 1.0f;
  while (true) {
    if (b & 1) r *= a;
    b /= 2;
    if (b == 0) break;
    a *= a;
  }
  return recip ? 1.0f / r : r;
}

float schlick(float cosine, float ref_idx) {  // :49-54
  float r0 = (1.0f - ref_idx) / (1.0f + ref_idx);
  r0 = r0 * r0;
  return r0 + (1.0f - r0) * powi(1.0f - cosine, 5);
}

// ---- shapes/hitable.rs ------------------------------------------------------
struct Hitable {
  virtual ~Hitable() {}
  virtual bool hit(Ray ray, float t_min, float t_max, HitRecord& rec) const = 0;
  virtual bool scatter(Ray ray, HitRecord& rec, ReflectRecord& rr, Rng& rng) const = 0;
};

// ---- shapes/sphere.rs -------------------------------------------------------
struct Sphere : Hitable {
  Vec3 center;
  float radius;
  uint32_t material;
  Vec3 color;
  float fuzz;
  bool hit(Ray ray, float t_min, float t_max, HitRecord& rec) const override {  // :23-51
    Vec3 origin_to_center = ray.origin() - center;
    float a = Vec3::dot(ray.direction(), ray.direction());
    float b = Vec3::dot(origin_to_center, ray.direction());
    float c = Vec3::dot(origin_to_center, origin_to_center) - radius * radius;
    float discriminant = b * b - a * c;
    if (discriminant > 0.0f) {
      float root_one = (-b - sqrtf(discriminant)) / a;
      if (root_one > t_min && root_one < t_max) {
        rec.t = root_one;
        rec.p = ray.point_at(root_one);
        rec.normal = (rec.p - center) / radius;
        return true;
      }
      float root_two = (-b + sqrtf(discriminant)) / a;
      if (root_two > t_min && root_two < t_max) {
        rec.t = root_two;
        rec.p = ray.point_at(root_two);
        rec.normal = (rec.p - center) / radius;
        return true;
      }
    }
    return false;
  }
  bool scatter(Ray ray, HitRecord& rec, ReflectRecord& rr, Rng& rng) const override {  // :53-70
    if (material == 0) return lambertian(rec, rr, rng);
    if (material == 1) return metal(ray, rec, rr, rng);
    if (material == 2) return dielectric(ray, rec, rr, rng);
    if (material == 3) return light(rec, rr, rng);
    return lambertian(rec, rr, rng);
  }
  bool lambertian(HitRecord& rec, ReflectRecord& rr, Rng& rng) const {  // :84-89
    Vec3 target = rec.p + rec.normal + random_in_unit_sphere(rng);
    rr.scattered = Ray(rec.p, target - rec.p);
    rr.attenuation = color;
    return true;
  }
  bool metal(Ray ray, HitRecord& rec, ReflectRecord& rr, Rng& rng) const {  // :91-105
    Vec3 reflected = reflect(ray.direction().unit_vector(), rec.normal);
    rr.scattered = Ray(rec.p, reflected + fuzz * random_in_unit_sphere(rng));
    rr.attenuation = color;
    return Vec3::dot(rr.scattered.direction(), rec.normal) > 0.0f;
  }
  bool dielectric(Ray ray, HitRecord& rec, ReflectRecord& rr, Rng& rng) const {  // :107-145
    const float ref_idx = 1.3f;
    Vec3 outward_normal = Vec3::zero();
    Vec3 reflected = reflect(ray.direction(), rec.normal);
    float ni_over_nt;
    rr.attenuation = color;
    Vec3 refracted = Vec3::zero();
    float reflect_prob;
    float cosine;
    if (Vec3::dot(ray.direction(), rec.normal) > 0.0f) {
      outward_normal = outward_normal - rec.normal;
      ni_over_nt = ref_idx;
      cosine = ref_idx * Vec3::dot(ray.direction(), rec.normal) / ray.direction().length();
    } else {
      outward_normal = rec.normal;
      ni_over_nt = 1.0f / ref_idx;
      cosine = -Vec3::dot(ray.direction(), rec.normal) / ray.direction().length();
    }
    if (refract(ray.direction(), outward_normal, ni_over_nt, refracted))
      reflect_prob = schlick(cosine, ref_idx);
    else
      reflect_prob = 1.0f;
    if (rng.gen_f32() < reflect_prob)
      rr.scattered = Ray(rec.p, reflected);
    else
      rr.scattered = Ray(rec.p, refracted);
    return true;
  }
  bool light(HitRecord& rec, ReflectRecord& rr, Rng& rng) const {  // :147-152
    Vec3 target = rec.p + rec.normal + random_in_unit_sphere(rng);
    rr.scattered = Ray(rec.p, target - rec.p);
    rr.attenuation = Vec3::one();
    return true;
  }
};

// ---- shapes/plane.rs --------------------------------------------------------
struct Plane : Hitable {
  Vec3 position, orientation, size;
  uint32_t material;
  Vec3 color;
  float fuzz;
  bool hit(Ray ray, float t_min, float t_max, HitRecord& rec) const override {  // :24-44
    float denom = Vec3::dot(orientation, ray.direction());
    if (denom > t_min && denom < t_max) {
      Vec3 plane_to_ray = position - ray.origin();
      rec.t = Vec3::dot(plane_to_ray, orientation) / denom;
      rec.p = ray.point_at(rec.t);
      if (rec.p.x > position.x - size.x && rec.p.x < position.x + size.x && rec.p.y > position.y - size.y &&
          rec.p.y < position.y + size.y && rec.p.z > position.z - size.z && rec.p.z < position.z + size.z) {
        rec.normal = orientation * -1.0f;
        return true;
      }
      return false;
    }
    return false;
  }
  bool scatter(Ray ray, HitRecord& rec, ReflectRecord& rr, Rng& rng) const override {  // :46-60
    if (material == 0) return lambertian(rec, rr, rng);
    if (material == 1) return metal(ray, rec, rr, rng);
    return lambertian(rec, rr, rng);
  }
  bool lambertian(HitRecord& rec, ReflectRecord& rr, Rng& rng) const {  // :101-106
    Vec3 target = rec.p + rec.normal + random_in_unit_sphere(rng);
    rr.scattered = Ray(rec.p, target - rec.p);
    rr.attenuation = color;
    return true;
  }
  bool metal(Ray ray, HitRecord& rec, ReflectRecord& rr, Rng& rng) const {  // :108-122
    Vec3 reflected = reflect(ray.direction().unit_vector(), rec.normal);
    rr.scattered = Ray(rec.p, reflected + fuzz * random_in_unit_sphere(rng));
    rr.attenuation = color;
    return Vec3::dot(rr.scattered.direction(), rec.normal) > 0.0f;
  }
};

// ---- shapes/aabb.rs, rectangle.rs stubs ---------------------------------------
struct Stub : Hitable {
  bool hit(Ray, float, float, HitRecord&) const override { return false; }
  bool scatter(Ray, HitRecord&, ReflectRecord&, Rng&) const override { return false; }
};

// ---- build-defined box, restated from its written spec ------
// Slabs per axis k: t0 = (lo_k - o_k) * (1/d_k), t1 = (hi_k - o_k) * (1/d_k) (the oriented
// box; the axis-aligned one computes them as Aabb::slabs_fma does, OR_BOX_FMA);
// near_k = fminf(t0, t1), far_k = fmaxf(t0, t1) (C99 fmin/fmax: NaN-ignoring);
// tn = fmaxf(fmaxf(near_x, near_y), near_z), tf = fminf(fminf(far_x, far_y), far_z).
// Hit iff tn < tf; then the near root if it is in (t_min, t_max), else the far root
// (Sphere::hit's two-root shape). Normal: outward face of the first axis (x, y, z)
// whose near value equals tn (entry, -sign(d_k)) or whose far value equals tf
// (exit, +sign(d_k)); sign(0) counts as negative. Scatter: Sphere::scatter's table.
struct BoxBase : Hitable {
  uint32_t material;
  Vec3 color;
  float fuzz;
  static float pick(Vec3 v, int k) { return k == 0 ? v.x : (k == 1 ? v.y : v.z); }
  static bool slabs(Vec3 lo, Vec3 hi, Vec3 o, Vec3 d, float t_min, float t_max, float& t, Vec3& n_local) {
    float t0[3], t1[3], nr[3], fr[3];
    for (int k = 0; k < 3; ++k) {
      const float inv = 1.0f / pick(d, k);
      t0[k] = (pick(lo, k) - pick(o, k)) * inv;
      t1[k] = (pick(hi, k) - pick(o, k)) * inv;
      nr[k] = fminf(t0[k], t1[k]);
      fr[k] = fmaxf(t0[k], t1[k]);
    }
    const float tn = fmaxf(fmaxf(nr[0], nr[1]), nr[2]);
    const float tf = fminf(fminf(fr[0], fr[1]), fr[2]);
    if (!(tn < tf)) return false;
    int k;
    float s;
    if (tn > t_min && tn < t_max) {
      t = tn;
      k = nr[0] == tn ? 0 : (nr[1] == tn ? 1 : 2);
      s = pick(d, k) > 0.0f ? -1.0f : 1.0f;
    } else if (tf > t_min && tf < t_max) {
      t = tf;
      k = fr[0] == tf ? 0 : (fr[1] == tf ? 1 : 2);
      s = pick(d, k) > 0.0f ? 1.0f : -1.0f;
    } else {
      return false;
    }
    n_local = Vec3();
    (k == 0 ? n_local.x : k == 1 ? n_local.y : n_local.z) = s;
    return true;
  }
  bool scatter(Ray ray, HitRecord& rec, ReflectRecord& rr, Rng& rng) const override {
    Sphere s;  // the sphere's material code (sphere.rs:53-152)
    s.material = material;
    s.color = color;
    s.fuzz = fuzz;
    return s.scatter(ray, rec, rr, rng);
  }
};

#ifndef OR_BOX_FMA
#define OR_BOX_FMA 1  // the box definition since round 6; 0: round 5's
#endif
struct Aabb : BoxBase {
  Vec3 mn, mx;
  // OR_BOX_FMA: the axis-aligned box's slab distances as fmaf(lo_k, inv_k, -(o_k * inv_k))
  // with inv_k = RN(1 / d_k) clamped to [-2^100, 2^100] (fmaxf, then fminf), the rest as
  // slabs() (the product's FR_BOX_FMA)
  static bool slabs_fma(Vec3 lo, Vec3 hi, Vec3 o, Vec3 d, float t_min, float t_max, float& t, Vec3& n_local) {
    float t0[3], t1[3], nr[3], fr[3];
    for (int k = 0; k < 3; ++k) {
      const float inv = fminf(fmaxf(1.0f / pick(d, k), -0x1p100f), 0x1p100f);
      const float oinv = pick(o, k) * inv;
      t0[k] = fmaf(pick(lo, k), inv, -oinv);
      t1[k] = fmaf(pick(hi, k), inv, -oinv);
      nr[k] = fminf(t0[k], t1[k]);
      fr[k] = fmaxf(t0[k], t1[k]);
    }
    const float tn = fmaxf(fmaxf(nr[0], nr[1]), nr[2]);
    const float tf = fminf(fminf(fr[0], fr[1]), fr[2]);
    if (!(tn < tf)) return false;
    int k;
    float s;
    if (tn > t_min && tn < t_max) {
      t = tn;
      k = nr[0] == tn ? 0 : (nr[1] == tn ? 1 : 2);
      s = pick(d, k) > 0.0f ? -1.0f : 1.0f;
    } else if (tf > t_min && tf < t_max) {
      t = tf;
      k = fr[0] == tf ? 0 : (fr[1] == tf ? 1 : 2);
      s = pick(d, k) > 0.0f ? 1.0f : -1.0f;
    } else {
      return false;
    }
    n_local = Vec3();
    (k == 0 ? n_local.x : k == 1 ? n_local.y : n_local.z) = s;
    return true;
  }
  bool hit(Ray ray, float t_min, float t_max, HitRecord& rec) const override {
    float t;
    Vec3 n;
    const bool h = OR_BOX_FMA ? slabs_fma(mn, mx, ray.origin(), ray.direction(), t_min, t_max, t, n)
                              : slabs(mn, mx, ray.origin(), ray.direction(), t_min, t_max, t, n);
    if (!h) return false;
    rec.t = t;
    rec.p = ray.point_at(t);
    rec.normal = n;
    return true;
  }
};

struct Obb : BoxBase {
  Vec3 center, ax[3], half;
  bool hit(Ray ray, float t_min, float t_max, HitRecord& rec) const override {
    const Vec3 oc = ray.origin() - center;
    const Vec3 d = ray.direction();
    const Vec3 ol(Vec3::dot(ax[0], oc), Vec3::dot(ax[1], oc), Vec3::dot(ax[2], oc));
    const Vec3 dl(Vec3::dot(ax[0], d), Vec3::dot(ax[1], d), Vec3::dot(ax[2], d));
    const Vec3 lo(-half.x, -half.y, -half.z);
    float t;
    Vec3 nl;
    if (!slabs(lo, half, ol, dl, t_min, t_max, t, nl)) return false;
    rec.t = t;
    rec.p = ray.point_at(t);
    // the local normal has one non-zero component s; world normal = s * that axis
    const int k = nl.x != 0.0f ? 0 : (nl.y != 0.0f ? 1 : 2);
    rec.normal = (nl.x + nl.y + nl.z) * ax[k];
    return true;
  }
};

// Build-defined triangle: Moller-Trumbore, f32, fixed order; the
// JSON triangle/circle/cylinder/tetrahedron meshes and tilted quads become lists of
// these. Normal: unit(cross(e1, e2)) by winding; for every material but dielectric it
// is turned to face the incoming ray (the raster meshes are double-faced).
struct Triangle : BoxBase {
  Vec3 v0, v1, v2;
  bool hit(Ray ray, float t_min, float t_max, HitRecord& rec) const override {
    const Vec3 e1 = v1 - v0, e2 = v2 - v0;
    const Vec3 d = ray.direction();
    const Vec3 pv = Vec3::cross(d, e2);
    const float inv_det = 1.0f / Vec3::dot(e1, pv);
    const Vec3 s = ray.origin() - v0;
    const float u = Vec3::dot(s, pv) * inv_det;
    const Vec3 qv = Vec3::cross(s, e1);
    const float v = Vec3::dot(d, qv) * inv_det;
    const float t = Vec3::dot(e2, qv) * inv_det;
    if (!(u >= 0.0f && v >= 0.0f && u + v <= 1.0f && t > t_min && t < t_max)) return false;
    rec.t = t;
    rec.p = ray.point_at(t);
    Vec3 n = Vec3::cross(e1, e2).unit_vector();
    if (material != 2u && Vec3::dot(n, d) > 0.0f) n = -1.0f * n;
    rec.normal = n;
    return true;
  }
};

// ---- cpu_ray_tracer/camera.rs -------------------------------------------------
const float PI = 3.14159265359f;  // :5

}  // namespace

extern "C" {

// Same field order as camera.rs:8-21 (checked against the product's fr_camera in tests)
typedef struct or_camera {
  float position[3], lower_left[3], horizontal[3], vertical[3], u[3], v[3], w[3];
  float aspect, lens_radius, focus_dist, radius, rotation;
} or_camera;

typedef struct or_prim {
  uint32_t kind, material;
  float color[3];
  float fuzz;
  float g[16];
} or_prim;

typedef struct or_counters {
  uint64_t segments, hits, samples, scatters;
} or_counters;
}

namespace {

struct Camera {
  Vec3 position, lower_left_corner, horizontal, vertical, u, v, w;
  float aspect, lens_radius, focus_dist, radius, rotation;

  void basis(Vec3 look_from, Vec3 look_at, Vec3 v_up, float v_fov, float aperture) {  // camera.rs:24-60
    float fd = (look_from - look_at).length();
    lens_radius = aperture / 2.0f;
    float theta = v_fov * PI / 180.0f;
    float half_height = tanf(theta / 2.0f);
    float half_width = aspect * half_height;
    position = look_from;
    w = (look_from - look_at).unit_vector();
    u = Vec3::cross(v_up, w).unit_vector();
    v = Vec3::cross(w, u);
    lower_left_corner = position - half_width * fd * u - half_height * fd * v - fd * w;
    horizontal = 2.0f * half_width * fd * u;
    vertical = 2.0f * half_height * fd * v;
  }
  Ray get_ray(float s, float t, Rng& rng) const {  // :62-72
    Vec3 rd = lens_radius * random_in_unit_circle(rng);
    Vec3 offset = rd.x * u + rd.y * v;
    return Ray(position + offset, lower_left_corner + s * horizontal + t * vertical - position - offset);
  }
  void orbit(Vec3 delta) {  // :97-122
    rotation += delta.x;
    radius += delta.z;
    position.x = radius * cosf(rotation);
    position.y += delta.y;
    position.z = radius * sinf(rotation);
    basis(position, Vec3(0.0f, 0.0f, 0.0f), Vec3(0.0f, 1.0f, 0.0f), 60.0f, 0.1f);
  }
  void translate(Vec3 delta) {  // :74-95
    position = position + delta;
    basis(position, Vec3(0.0f, 0.0f, -1.0f), Vec3(0.0f, 1.0f, 0.0f), 60.0f, 0.1f);
  }
  void to_c(or_camera* c) const {
    const Vec3* src[7] = {&position, &lower_left_corner, &horizontal, &vertical, &u, &v, &w};
    float* dst[7] = {c->position, c->lower_left, c->horizontal, c->vertical, c->u, c->v, c->w};
    for (int i = 0; i < 7; ++i) {
      dst[i][0] = src[i]->x;
      dst[i][1] = src[i]->y;
      dst[i][2] = src[i]->z;
    }
    c->aspect = aspect;
    c->lens_radius = lens_radius;
    c->focus_dist = focus_dist;
    c->radius = radius;
    c->rotation = rotation;
  }
  void from_c(const or_camera* c) {
    Vec3* dst[7] = {&position, &lower_left_corner, &horizontal, &vertical, &u, &v, &w};
    const float* src[7] = {c->position, c->lower_left, c->horizontal, c->vertical, c->u, c->v, c->w};
    for (int i = 0; i < 7; ++i) *dst[i] = Vec3(src[i][0], src[i][1], src[i][2]);
    aspect = c->aspect;
    lens_radius = c->lens_radius;
    focus_dist = c->focus_dist;
    radius = c->radius;
    rotation = c->rotation;
  }
};

// one cache line per thread's counters: they are bumped on every segment, and adjacent
// per-thread counters would share lines between cores (false sharing cost the threaded
// oracle about 3x at 16 threads)
struct alignas(64) Counters {
  uint64_t segments = 0, hits = 0, scatters = 0;
};

// ---- cpu_ray_tracer/tracer.rs:189-219 ---------------------------------------
Vec3 get_color(Ray ray, const std::vector<std::unique_ptr<Hitable>>& objects, uint32_t depth, uint32_t max_depth,
               Rng& rng, Counters& cnt) {
  ++cnt.segments;
  HitRecord hit_record;
  const float t_min = 0.001f;
  float closest_so_far = 3.40282347e+38f;  // f32::MAX
  const Hitable* temp_obj = nullptr;
  for (const auto& obj : objects) {
    if (obj->hit(ray, t_min, closest_so_far, hit_record)) {
      closest_so_far = hit_record.t;
      temp_obj = obj.get();
    }
  }
  if (temp_obj) {
    ++cnt.hits;
    ReflectRecord reflect_record;
    if (depth < max_depth && temp_obj->scatter(ray, hit_record, reflect_record, rng)) {
      ++cnt.scatters;
      return reflect_record.attenuation * get_color(reflect_record.scattered, objects, depth + 1, max_depth, rng, cnt);
    }
    return Vec3::zero();
  }
  Vec3 unit_direction = ray.direction().unit_vector();
  float t = 0.5f * (unit_direction.y + 1.0f);
  return (1.0f - t) * Vec3(1.0f, 1.0f, 1.0f) + t * Vec3(0.5f, 0.7f, 1.0f);
}

std::vector<std::unique_ptr<Hitable>> build(const or_prim* prims, uint32_t n) {
  std::vector<std::unique_ptr<Hitable>> out;
  for (uint32_t i = 0; i < n; ++i) {
    const or_prim& p = prims[i];
    const Vec3 color(p.color[0], p.color[1], p.color[2]);
    switch (p.kind) {
      case 0: {
        auto s = std::make_unique<Sphere>();
        s->center = Vec3(p.g[0], p.g[1], p.g[2]);
        s->radius = p.g[3];
        s->material = p.material;
        s->color = color;
        s->fuzz = p.fuzz;
        out.push_back(std::move(s));
        break;
      }
      case 1: {
        auto s = std::make_unique<Plane>();
        s->position = Vec3(p.g[0], p.g[1], p.g[2]);
        s->orientation = Vec3(p.g[3], p.g[4], p.g[5]);
        s->size = Vec3(p.g[6], p.g[7], p.g[8]);
        s->material = p.material;
        s->color = color;
        s->fuzz = p.fuzz;
        out.push_back(std::move(s));
        break;
      }
      case 2: {
        auto s = std::make_unique<Aabb>();
        s->mn = Vec3(p.g[0], p.g[1], p.g[2]);
        s->mx = Vec3(p.g[3], p.g[4], p.g[5]);
        s->material = p.material;
        s->color = color;
        s->fuzz = p.fuzz;
        out.push_back(std::move(s));
        break;
      }
      case 3: {
        auto s = std::make_unique<Obb>();
        s->center = Vec3(p.g[0], p.g[1], p.g[2]);
        s->ax[0] = Vec3(p.g[3], p.g[4], p.g[5]);
        s->ax[1] = Vec3(p.g[6], p.g[7], p.g[8]);
        s->ax[2] = Vec3(p.g[9], p.g[10], p.g[11]);
        s->half = Vec3(p.g[12], p.g[13], p.g[14]);
        s->material = p.material;
        s->color = color;
        s->fuzz = p.fuzz;
        out.push_back(std::move(s));
        break;
      }
      case 5: {
        auto s = std::make_unique<Triangle>();
        s->v0 = Vec3(p.g[0], p.g[1], p.g[2]);
        s->v1 = Vec3(p.g[3], p.g[4], p.g[5]);
        s->v2 = Vec3(p.g[6], p.g[7], p.g[8]);
        s->material = p.material;
        s->color = color;
        s->fuzz = p.fuzz;
        out.push_back(std::move(s));
        break;
      }
      default: out.push_back(std::make_unique<Stub>());
    }
  }
  return out;
}

uint8_t as_u8(float v) {  // Rust `f32 as u8`: saturating, NaN -> 0, truncation
  if (!(v > 0.0f)) return 0;
  if (v >= 255.0f) return 255;
  return uint8_t(v);
}

}  // namespace

extern "C" {

int oracle_abi_version(void) { return 1; }

// Camera::new generalised to an arbitrary look-from/look-at
void oracle_camera_look(const float from[3], const float at[3], const float vup[3], float vfov, float aperture,
                        uint32_t width, uint32_t height, or_camera* out) {
  Camera c;
  c.aspect = float(width) / float(height);
  c.basis(Vec3(from[0], from[1], from[2]), Vec3(at[0], at[1], at[2]), Vec3(vup[0], vup[1], vup[2]), vfov,
          aperture);
  c.focus_dist = 2.0f;
  c.radius = 5.0f;
  c.rotation = 0.0f;
  c.to_c(out);
}

void oracle_camera_new(uint32_t width, uint32_t height, or_camera* out) {  // camera.rs:24-60
  const float from[3] = {0.0f, 0.0f, 1.0f}, at[3] = {0.0f, 0.0f, 0.0f}, up[3] = {0.0f, 1.0f, 0.0f};
  oracle_camera_look(from, at, up, 60.0f, 0.1f, width, height, out);
}

void oracle_camera_orbit(or_camera* cam, const float delta[3]) {
  Camera c;
  c.from_c(cam);
  c.orbit(Vec3(delta[0], delta[1], delta[2]));
  c.to_c(cam);
}

void oracle_camera_translate(or_camera* cam, const float delta[3]) {
  Camera c;
  c.from_c(cam);
  c.translate(Vec3(delta[0], delta[1], delta[2]));
  c.to_c(cam);
}

void oracle_rng_stream(uint64_t seed, uint32_t pixel, uint32_t sample, uint32_t n, uint32_t* out) {
  Rng r(seed, pixel, sample);
  for (uint32_t i = 0; i < n; ++i) out[i] = r.next_u32();
}

// Vec3 primitives for the reference's own KATs (primitives.rs:159-255):
// op 0 length_squared(a), 1 length(a), 2 dot(a,b), 3 cross(a,b), 4 a+b, 5 a-b,
// 6 a*s (s = b[0]), 7 a*b, 8 a/s (s = b[0]), 9 unit_vector(a), 10 reflect(a,b),
// 11 refract(a, b, ni = b... see tests), 12 schlick(a[0], a[1]); out[3]
void oracle_vec3(int op, const float a[3], const float b[3], float out[3]) {
  const Vec3 va(a[0], a[1], a[2]), vb(b[0], b[1], b[2]);
  Vec3 r;
  switch (op) {
    case 0: r.x = va.length_squared(); break;
    case 1: r.x = va.length(); break;
    case 2: r.x = Vec3::dot(va, vb); break;
    case 3: r = Vec3::cross(va, vb); break;
    case 4: r = va + vb; break;
    case 5: r = va - vb; break;
    case 6: r = va * b[0]; break;
    case 7: r = va * vb; break;
    case 8: r = va / b[0]; break;
    case 9: r = va.unit_vector(); break;
    case 10: r = reflect(va, vb); break;
    case 12: r.x = schlick(a[0], a[1]); break;
    default: break;
  }
  out[0] = r.x;
  out[1] = r.y;
  out[2] = r.z;
}

// refract(v, n, ni) -> (ok, refracted)
int oracle_refract(const float v[3], const float n[3], float ni, float out[3]) {
  Vec3 r;
  const bool ok = refract(Vec3(v[0], v[1], v[2]), Vec3(n[0], n[1], n[2]), ni, r);
  out[0] = r.x;
  out[1] = r.y;
  out[2] = r.z;
  return ok ? 1 : 0;
}

// One ray through the closest-hit loop (tracer.rs:190-200) for analytic KATs.
// Returns the winning index or -1; fills t, p, normal of the shared record.
int oracle_closest_hit(const or_prim* prims, uint32_t n, const float o[3], const float d[3], float rec[7]) {
  auto objs = build(prims, n);
  HitRecord hr;
  float closest = 3.40282347e+38f;
  int best = -1;
  const Ray ray(Vec3(o[0], o[1], o[2]), Vec3(d[0], d[1], d[2]));
  for (uint32_t i = 0; i < n; ++i)
    if (objs[i]->hit(ray, 0.001f, closest, hr)) {
      closest = hr.t;
      best = int(i);
    }
  rec[0] = hr.t;
  rec[1] = hr.p.x;
  rec[2] = hr.p.y;
  rec[3] = hr.p.z;
  rec[4] = hr.normal.x;
  rec[5] = hr.normal.y;
  rec[6] = hr.normal.z;
  return best;
}

// save_image's loop (tracer.rs:160-187) over the rows of one shard
// (strips of 8 rows, strip k -> shard k % shard_count), keeping every
// `row_step`-th of those rows (1 = all) and in them every `col_step`-th pixel
// (1 = all). Parallel over `threads` in chunks of 32 pixels of a row (the render_mt
// shape, tracer.rs:83-134, without its per-pixel scene rebuild). Writes means and u8
// for the pixels it renders; returns the number of rows.
int64_t oracle_render_rows(const or_prim* prims, uint32_t n, const or_camera* cam, uint32_t width, uint32_t height,
                           uint32_t spp, uint32_t max_depth, uint64_t seed, const uint32_t* row_list,
                           uint32_t n_rows, uint32_t col_step, int threads, float* out_mean, uint8_t* out_u8,
                           or_counters* counters);

int64_t oracle_render(const or_prim* prims, uint32_t n, const or_camera* cam, uint32_t width, uint32_t height,
                      uint32_t spp, uint32_t max_depth, uint64_t seed, uint32_t shard_index, uint32_t shard_count,
                      uint32_t row_step, uint32_t col_step, int threads, float* out_mean, uint8_t* out_u8,
                      or_counters* counters) {
  if (!cam || width == 0 || height == 0 || shard_count == 0 || shard_index >= shard_count || row_step == 0 ||
      col_step == 0)
    return -1;
  std::vector<uint32_t> rows;
  uint32_t kept = 0;
  for (uint32_t y = 0; y < height; ++y) {
    if ((y / 8) % shard_count != shard_index) continue;
    if (kept++ % row_step == 0) rows.push_back(y);
  }
  return oracle_render_rows(prims, n, cam, width, height, spp, max_depth, seed, rows.data(),
                            static_cast<uint32_t>(rows.size()), col_step, threads, out_mean, out_u8, counters);
}

// The same loop over an explicit list of image rows (each < height).
int64_t oracle_render_rows(const or_prim* prims, uint32_t n, const or_camera* cam, uint32_t width, uint32_t height,
                           uint32_t spp, uint32_t max_depth, uint64_t seed, const uint32_t* row_list,
                           uint32_t n_rows, uint32_t col_step, int threads, float* out_mean, uint8_t* out_u8,
                           or_counters* counters) {
  if (!cam || width == 0 || height == 0 || col_step == 0 || (n_rows && !row_list)) return -1;
  for (uint32_t i = 0; i < n_rows; ++i)
    if (row_list[i] >= height) return -1;
  const std::vector<uint32_t> rows(row_list, row_list + n_rows);
  const auto objects = build(prims, n);
  Camera camera;
  camera.from_c(cam);
  const uint32_t cols = (width + col_step - 1) / col_step;  // pixels x = 0, col_step, ...
  const uint32_t chunk = 32, chunks = (cols + chunk - 1) / chunk;
  if (threads < 1) threads = 1;
  std::atomic<size_t> next{0};
  std::vector<Counters> cnts(threads);
  auto work = [&](int tid) {
    Counters cnt;  // thread-local while rendering, stored once at the end
    for (size_t wi; (wi = next.fetch_add(1)) < rows.size() * chunks;) {
      const uint32_t y = rows[wi / chunks];
      const uint32_t c0 = static_cast<uint32_t>(wi % chunks) * chunk;
      for (uint32_t c = c0; c < c0 + chunk && c < cols; ++c) {
        const uint32_t x = c * col_step;
        const uint32_t pixel = y * width + x;
        Vec3 col = Vec3::zero();
        Rng rng(seed, pixel, 0);
        for (uint32_t s = 0; s < spp; ++s) {
          // samples come in streams of 16 (4 in the last block); each draws in order
          uint32_t key;
          if (stream_start(s, spp, key)) rng = Rng(seed, pixel, key);
          const float u = (float(x) + rng.gen_f32()) / float(width);
          const float v = (float(height - y) + rng.gen_f32()) / float(height);
          const Ray ray = camera.get_ray(u, v, rng);
          col = col + get_color(ray, objects, 0, max_depth, rng, cnt);
        }
        col = col / float(spp);
        const size_t idx = size_t(pixel) * 3;
        if (out_mean) {
          out_mean[idx] = col.x;
          out_mean[idx + 1] = col.y;
          out_mean[idx + 2] = col.z;
        }
        if (out_u8) {
          const Vec3 g(sqrtf(col.r()), sqrtf(col.g()), sqrtf(col.b()));  // :178
          out_u8[idx] = as_u8(g.r() * 255.0f);
          out_u8[idx + 1] = as_u8(g.g() * 255.0f);
          out_u8[idx + 2] = as_u8(g.b() * 255.0f);
        }
      }
    }
    cnts[tid] = cnt;
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& t : pool) t.join();
  if (counters) {
    memset(counters, 0, sizeof(*counters));
    for (const auto& c : cnts) {
      counters->segments += c.segments;
      counters->hits += c.hits;
      counters->scatters += c.scatters;
    }
    counters->samples = uint64_t(rows.size()) * cols * spp;
  }
  return int64_t(rows.size());
}

// save_image_mt (tracer.rs:136-158) over render_mt (tracer.rs:83-134), in their
// shape: `sample` passes; each pass renders 4 row bands of t_height = H/4 rows (band
// t_id covers image rows from the top in the order 3, 2, 1, 0) with
// v = ((t_height - y) + r) / H + t_id * 0.25, gamma-corrects and quantises every pixel
// to u8, and the passes are averaged as acc += u8 / sample in f32, then `as u8`. Rows
// past 4 * t_height are never written (0). A pixel's passes draw from the build's
// streams exactly as save_image's samples do (stream_start of (seed, pixel)), so the
// per-pixel stream state is carried from pass to pass.
int oracle_render_mt(const or_prim* prims, uint32_t n, const or_camera* cam, uint32_t width, uint32_t height,
                     uint32_t sample, uint32_t max_depth, uint64_t seed, float* out_acc, uint8_t* out_u8,
                     or_counters* counters) {
  if (!cam || width == 0 || height == 0 || sample == 0 || !out_acc || !out_u8) return -1;
  const auto objects = build(prims, n);
  Camera camera;
  camera.from_c(cam);
  const uint32_t NTHREADS = 4;
  const uint32_t t_height = height / NTHREADS;
  const float t_offset = 1.0f / float(NTHREADS);
  std::vector<float> acc(size_t(width) * height * 3, 0.0f);
  std::vector<Rng> streams(size_t(width) * height, Rng(seed, 0, 0));
  Counters cnt;
  for (uint32_t pass = 0; pass < sample; ++pass) {
    std::vector<uint8_t> pixels(size_t(width) * height * 3, 0);  // render_mt's result, bands stacked
    for (uint32_t t_id = 0; t_id < NTHREADS; ++t_id) {
      for (uint32_t y = 0; y < t_height; ++y) {
        for (uint32_t x = 0; x < width; ++x) {
          const uint32_t row = (NTHREADS - 1 - t_id) * t_height + y;  // ids sorted descending (:122-127)
          const uint32_t pixel = row * width + x;
          Rng& rng = streams[pixel];
          uint32_t key;
          if (stream_start(pass, sample, key)) rng = Rng(seed, pixel, key);
          const float u = (float(x) + rng.gen_f32()) / float(width);
          float v = (float(t_height - y) + rng.gen_f32()) / float(height);
          v += float(t_id) * t_offset;
          const Ray ray = camera.get_ray(u, v, rng);
          const Vec3 color = get_color(ray, objects, 0, max_depth, rng, cnt);
          const size_t index = size_t(pixel) * 3;
          pixels[index] = as_u8(sqrtf(color.r()) * 255.0f);
          pixels[index + 1] = as_u8(sqrtf(color.g()) * 255.0f);
          pixels[index + 2] = as_u8(sqrtf(color.b()) * 255.0f);
        }
      }
    }
    const size_t filled = size_t(width) * t_height * NTHREADS * 3;
    for (size_t k = 0; k < filled; ++k) acc[k] += float(pixels[k]) / float(sample);  // :141-144
  }
  for (size_t k = 0; k < acc.size(); ++k) {
    out_acc[k] = acc[k];
    out_u8[k] = as_u8(acc[k]);
  }
  if (counters) {
    counters->segments = cnt.segments;
    counters->hits = cnt.hits;
    counters->scatters = cnt.scatters;
    counters->samples = uint64_t(width) * t_height * NTHREADS * sample;
  }
  return 0;
}

}  // extern "C"
