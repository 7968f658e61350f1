// scene.cpp — host side of libforma_rt: error state, the tracer camera
// (cpu_ray_tracer/camera.rs), the reference's built-in object lists
// (cpu_ray_tracer/scenes.rs), the scenes/*.json -> tracer primitive mapping
// (DESIGN.md §3), and Hitable::translate/rotate.
//
// Compiled with g++ -ffp-contract=off: camera setup is the only place that uses
// tan/sin/cos, and it runs on the host exactly once per frame.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>

#include "internal.h"
#include "json_min.h"
#include "rt_core.h"

namespace fr {

static thread_local std::string g_last_error;

int set_error(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
  return code;
}

namespace {

const float kPi = 3.14159265359f;  // camera.rs:5

V3 from_arr(const float a[3]) { return V3{a[0], a[1], a[2]}; }
void to_arr(V3 v, float a[3]) {
  a[0] = v.x;
  a[1] = v.y;
  a[2] = v.z;
}

// The basis update shared by Camera::new / translate / orbit (camera.rs:24-60,
// 74-95, 97-122): focus_dist = |from - at|, lens_radius = aperture / 2.
void camera_basis(fr_camera* c, V3 from, V3 at, V3 vup, float vfov, float aperture) {
  const float focus_dist = length(sub(from, at));
  c->lens_radius = aperture / 2.0f;
  const float theta = vfov * kPi / 180.0f;
  const float half_height = tanf(theta / 2.0f);
  const float half_width = c->aspect * half_height;
  const V3 w = unit(sub(from, at));
  const V3 u = unit(cross(vup, w));
  const V3 v = cross(w, u);
  // position - hw*fd*u - hh*fd*v - fd*w, left to right
  const V3 llc = sub(sub(sub(from, scl(half_width * focus_dist, u)), scl(half_height * focus_dist, v)),
                     scl(focus_dist, w));
  to_arr(from, c->position);
  to_arr(llc, c->lower_left);
  to_arr(scl(2.0f * half_width * focus_dist, u), c->horizontal);
  to_arr(scl(2.0f * half_height * focus_dist, v), c->vertical);
  to_arr(u, c->u);
  to_arr(v, c->v);
  to_arr(w, c->w);
}

fr_prim make_sphere(V3 c, float r, uint32_t mat, V3 color, float fuzz) {
  fr_prim p;
  memset(&p, 0, sizeof(p));
  p.kind = FR_SPHERE;
  p.material = mat;
  to_arr(color, p.color);
  p.fuzz = fuzz;
  p.g[0] = c.x;
  p.g[1] = c.y;
  p.g[2] = c.z;
  p.g[3] = r;
  return p;
}

fr_prim make_plane(V3 pos, V3 orient, V3 size, uint32_t mat, V3 color, float fuzz) {
  fr_prim p;
  memset(&p, 0, sizeof(p));
  p.kind = FR_PLANE;
  p.material = mat;
  to_arr(color, p.color);
  p.fuzz = fuzz;
  to_arr(pos, p.g);
  to_arr(orient, p.g + 3);
  to_arr(size, p.g + 6);
  return p;
}

V3 sqrt3(V3 a) { return V3{sqrtf(a.x), sqrtf(a.y), sqrtf(a.z)}; }  // primitives.rs:74-76

// cpu_ray_tracer/scenes.rs:6-39
std::vector<fr_prim> simple_scene() {
  std::vector<fr_prim> o;
  o.push_back(make_plane(mk(-1, 0, 0), mk(0, 0, 0), scl(5.0f, mk(1, 1, 1)), 1, mk(1.0f, 0.3f, 0.3f), 0.05f));
  o.push_back(make_sphere(mk(-0.5f, 0, 0), 0.5f, 0, mk(0.0f, 0.66f, 0.13f), 0.0f));
  o.push_back(make_sphere(mk(0.5f, 0, 0), 0.5f, 0, mk(0.7f, 0.43f, 0.0f), 0.0f));
  o.push_back(make_sphere(mk(0, -1000.5f, 0), 1000.0f, 0, mk(0.3f, 0.3f, 0.3f), 1.0f));
  return o;
}

// scenes.rs:41-108 (only the uncommented plane)
std::vector<fr_prim> plane_scene() {
  std::vector<fr_prim> o;
  o.push_back(make_plane(mk(-1, 0, 0), mk(0, 0, 0), scl(100.0f, mk(1, 1, 1)), 1, mk(0.1f, 0.9f, 0.1f), 0.0f));
  return o;
}

// scenes.rs:110-156
std::vector<fr_prim> objects_scene() {
  std::vector<fr_prim> o;
  o.push_back(make_sphere(mk(0, 0, -1), 0.5f, 0, mk(0.5f, 0.1f, 0.1f), 0.0f));
  o.push_back(make_sphere(mk(1, 0, -1), 0.5f, 1, mk(0.9f, 0.9f, 0.9f), 0.2f));
  o.push_back(make_sphere(mk(1, 0, -3), 0.5f, 1, mk(1.0f, 1.0f, 1.0f), 1.0f));
  o.push_back(make_sphere(mk(-1, -0.0f, -1), 0.5f, 2, sqrt3(sqrt3(sqrt3(mk(0.1f, 0.5f, 0.1f)))), 0.2f));
  o.push_back(make_sphere(mk(0, 0, 1), 0.5f, 2, sqrt3(sqrt3(sqrt3(mk(0.5f, 0.5f, 0.3f)))), 0.2f));
  o.push_back(make_sphere(mk(0, -100.5f, -1), 100.0f, 0, mk(0.1f, 0.3f, 0.9f), 0.0f));
  return o;
}

// ---- JSON mapping ----------------------------------------------------------

// CP0 palette, color_utils.rs:101-109
const float kCP0[4][3] = {
    {0.263f, 0.208f, 0.655f}, {1.000f, 0.498f, 0.243f}, {1.000f, 0.965f, 0.914f}, {0.502f, 0.769f, 0.914f}};

struct Axes {
  V3 x, y, z;  // images of the local unit axes (columns of the rotation)
};

// glam's quaternion -> rotation axes, in f32 (used by the TRS model matrix,
// primitives/primitive.rs:65-69)
Axes quat_axes(float x, float y, float z, float w) {
  const float x2 = x + x, y2 = y + y, z2 = z + z;
  const float xx = x * x2, xy = x * y2, xz = x * z2;
  const float yy = y * y2, yz = y * z2, zz = z * z2;
  const float wx = w * x2, wy = w * y2, wz = w * z2;
  Axes a;
  a.x = V3{1.0f - (yy + zz), xy + wz, xz - wy};
  a.y = V3{xy - wz, 1.0f - (xx + zz), yz + wx};
  a.z = V3{xz + wy, yz - wx, 1.0f - (xx + yy)};
  return a;
}

const float kSnap = 1e-5f;

// Snap one component to {-1, 0, +1}; returns false if it is none of them.
bool snap1(float v, float& out) {
  if (fabsf(v) < kSnap) {
    out = 0.0f;
    return true;
  }
  if (fabsf(fabsf(v) - 1.0f) < kSnap) {
    out = v > 0.0f ? 1.0f : -1.0f;
    return true;
  }
  return false;
}

// If the rotation is a signed permutation, fill perm[j] = world axis of local axis j
// and sign[j], and return true.
bool signed_permutation(const Axes& a, int perm[3], float sign[3]) {
  const V3 cols[3] = {a.x, a.y, a.z};
  int used = 0;
  for (int j = 0; j < 3; ++j) {
    float s[3];
    if (!snap1(cols[j].x, s[0]) || !snap1(cols[j].y, s[1]) || !snap1(cols[j].z, s[2])) return false;
    int nz = 0, at = -1;
    for (int i = 0; i < 3; ++i)
      if (s[i] != 0.0f) {
        ++nz;
        at = i;
      }
    if (nz != 1 || (used & (1 << at))) return false;
    used |= 1 << at;
    perm[j] = at;
    sign[j] = s[at];
  }
  return true;
}

bool num_f32(const json::Value* v, float& out) {
  if (!v || v->type != json::Value::Number) return false;
  out = strtof(v->text.c_str(), nullptr);
  return true;
}

bool vec3_of(const json::Value* v, V3& out) {
  if (!v || v->type != json::Value::Object) return false;
  return num_f32(v->get("x"), out.x) && num_f32(v->get("y"), out.y) && num_f32(v->get("z"), out.z);
}

bool quat_of(const json::Value* v, float q[4]) {
  if (!v || v->type != json::Value::Object) return false;
  return num_f32(v->get("x"), q[0]) && num_f32(v->get("y"), q[1]) && num_f32(v->get("z"), q[2]) &&
         num_f32(v->get("w"), q[3]);
}

// basics/scene.rs:59-80 material names -> tracer material
int material_of(const json::Value& obj, uint32_t& mat, V3& color, float& fuzz, int index) {
  const json::Value* m = obj.get("material");
  if (!m || m->type != json::Value::String)
    return set_error(FR_EPARSE, "objects[%d]: missing string field 'material'", index);
  int pal = 0;
  if (m->text == "EqualizerMaterial")
    pal = 1;
  else if (m->text == "WaveMaterial")
    pal = 2;
  else if (m->text == "Texture" || m->text == "UnlitColorMaterial")
    pal = 3;
  else if (m->text == "DiffuseTexture")
    return set_error(FR_EPARSE, "objects[%d]: material 'DiffuseTexture' is todo!() in basics/scene.rs:74",
                     index);
  mat = FR_LAMBERTIAN;
  color = V3{kCP0[pal][0], kCP0[pal][1], kCP0[pal][2]};
  fuzz = 0.0f;
  // build-only extension: "rt": {"material": ..., "color": [r,g,b], "fuzz": f}
  const json::Value* rt = obj.get("rt");
  if (rt) {
    if (rt->type != json::Value::Object) return set_error(FR_EPARSE, "objects[%d]: 'rt' must be an object", index);
    const json::Value* rm = rt->get("material");
    if (rm) {
      if (rm->type != json::Value::String) return set_error(FR_EPARSE, "objects[%d]: rt.material", index);
      if (rm->text == "lambertian")
        mat = FR_LAMBERTIAN;
      else if (rm->text == "metal")
        mat = FR_METAL;
      else if (rm->text == "dielectric")
        mat = FR_DIELECTRIC;
      else if (rm->text == "light")
        mat = FR_LIGHT;
      else
        return set_error(FR_EPARSE, "objects[%d]: unknown rt.material '%s'", index, rm->text.c_str());
    }
    const json::Value* rc = rt->get("color");
    if (rc) {
      if (rc->type != json::Value::Array || rc->items.size() != 3 || !num_f32(&rc->items[0], color.x) ||
          !num_f32(&rc->items[1], color.y) || !num_f32(&rc->items[2], color.z))
        return set_error(FR_EPARSE, "objects[%d]: rt.color must be [r, g, b]", index);
    }
    const json::Value* rf = rt->get("fuzz");
    if (rf && !num_f32(rf, fuzz)) return set_error(FR_EPARSE, "objects[%d]: rt.fuzz", index);
  }
  return FR_OK;
}

// ---- meshes as triangle lists (primitives/*.rs vertex and index tables) ----------

struct Mesh {
  std::vector<V3> v;        // local vertex positions
  std::vector<uint32_t> i;  // triangles, three indices each
};

// f32 sector angle as the mesh generators write it: `i as f32 * 2.0 * PI / n as f32`
// (circle.rs:67, cylinder.rs:76), and its cosine / sine rounded from double
float sector_angle(uint32_t i, uint32_t n) {
  const float kPiF = 3.14159265358979323846f;  // std::f32::consts::PI
  return ((static_cast<float>(i) * 2.0f) * kPiF) / static_cast<float>(n);
}
float cos_rn(float a) { return static_cast<float>(cos(static_cast<double>(a))); }
float sin_rn(float a) { return static_cast<float>(sin(static_cast<double>(a))); }

Mesh mesh_triangle() {  // triangle.rs:6-13
  return Mesh{{V3{0.0f, 0.5f, 0.0f}, V3{-0.5f, -0.5f, 0.0f}, V3{0.5f, -0.5f, 0.0f}}, {0, 1, 2}};
}

Mesh mesh_quad() {  // quad.rs:7-17
  return Mesh{{V3{-0.5f, -0.5f, 0.0f}, V3{0.5f, -0.5f, 0.0f}, V3{0.5f, 0.5f, 0.0f}, V3{-0.5f, 0.5f, 0.0f}},
              {0, 1, 2, 2, 3, 0}};
}

Mesh mesh_tetrahedron() {  // tetrahedron.rs:13-32 (X = 1)
  const float X = 1.0f;
  return Mesh{{V3{X, X, -X}, V3{X, -X, X}, V3{-X, X, X}, V3{-X, X, X}, V3{-X, -X, -X}, V3{X, X, -X},
               V3{-X, X, X}, V3{X, -X, X}, V3{-X, -X, -X}, V3{X, X, -X}, V3{-X, -X, -X}, V3{X, -X, X}},
              {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11}};
}

Mesh mesh_circle() {  // circle.rs:64-107: 36 sectors, radius 0.5, z = 0, centre last
  const uint32_t n = 36;
  Mesh m;
  for (uint32_t k = 0; k < n; ++k) {
    const float a = sector_angle(k, n);
    m.v.push_back(V3{0.5f * cos_rn(a), 0.5f * sin_rn(a), 0.0f});
  }
  m.v.push_back(V3{0.0f, 0.0f, 0.0f});
  for (uint32_t k = 0; k < n; ++k) {
    m.i.push_back(k);
    m.i.push_back((k + 1) % n);
    m.i.push_back(n);
  }
  return m;
}

Mesh mesh_cylinder(uint32_t n) {  // cylinder.rs:72-174 with sector_count 30 (basics/scene.rs:90)
  Mesh m;
  const float ys[2] = {0.5f, -0.5f};
  for (int cap = 0; cap < 2; ++cap) {  // top ring + centre, bottom ring + centre
    for (uint32_t k = 0; k < n; ++k) {
      const float a = sector_angle(k, n);
      m.v.push_back(V3{0.5f * cos_rn(a), ys[cap], 0.5f * sin_rn(a)});
    }
    m.v.push_back(V3{0.0f, ys[cap], 0.0f});
  }
  for (int ring = 0; ring < 2; ++ring)  // side rings (same positions, own normals upstream)
    for (uint32_t k = 0; k < n; ++k) {
      const float a = sector_angle(k, n);
      m.v.push_back(V3{0.5f * cos_rn(a), ys[ring], 0.5f * sin_rn(a)});
    }
  for (uint32_t k = 0; k < n; ++k) {  // top
    m.i.insert(m.i.end(), {k, (k + 1) % n, n});
  }
  const uint32_t off = n + 1;
  for (uint32_t k = 0; k < n; ++k) {  // bottom
    m.i.insert(m.i.end(), {(k + 1) % n + off, k + off, n + off});
  }
  const uint32_t side = 2 * (n + 1);
  for (uint32_t k = 0; k < n; ++k) {  // sides, two triangles per sector
    m.i.insert(m.i.end(), {(k + 1) % n + side, k + side, (k + 1) % n + side + n});
    m.i.insert(m.i.end(), {k + side + n, (k + 1) % n + side + n, k + side});
  }
  return m;
}

// Model transform of one vertex, f32, in this order:
// w = ((ax.x (s.x l.x) + ax.y (s.y l.y)) + ax.z (s.z l.z)) + pos, per component
V3 to_world(const Axes& ax, V3 s, V3 pos, V3 l) {
  const float sx = s.x * l.x, sy = s.y * l.y, sz = s.z * l.z;
  return V3{((ax.x.x * sx + ax.y.x * sy) + ax.z.x * sz) + pos.x, ((ax.x.y * sx + ax.y.y * sy) + ax.z.y * sz) + pos.y,
            ((ax.x.z * sx + ax.y.z * sy) + ax.z.z * sz) + pos.z};
}

void append_mesh(const Mesh& m, const Axes& ax, V3 scale, V3 pos, const fr_prim& base, std::vector<fr_prim>& out) {
  std::vector<V3> w(m.v.size());
  for (size_t k = 0; k < m.v.size(); ++k) w[k] = to_world(ax, scale, pos, m.v[k]);
  for (size_t t = 0; t + 2 < m.i.size(); t += 3) {
    fr_prim p = base;
    p.kind = FR_TRIANGLE;
    to_arr(w[m.i[t]], p.g);
    to_arr(w[m.i[t + 1]], p.g + 3);
    to_arr(w[m.i[t + 2]], p.g + 6);
    out.push_back(p);
  }
}

// One JSON object -> its tracer primitives, appended to `list` (one for sphere / cube /
// axis-aligned quad, a triangle list for the other meshes).
int map_object(const json::Value& obj, int index, std::vector<fr_prim>& list) {
  if (obj.type != json::Value::Object) return set_error(FR_EPARSE, "objects[%d] is not an object", index);
  const json::Value* mesh = obj.get("mesh");
  if (!mesh || mesh->type != json::Value::String)
    return set_error(FR_EPARSE, "objects[%d]: missing string field 'mesh'", index);
  V3 pos, scale;
  float q[4];
  if (!vec3_of(obj.get("position"), pos)) return set_error(FR_EPARSE, "objects[%d]: bad 'position'", index);
  if (!quat_of(obj.get("rotation"), q)) return set_error(FR_EPARSE, "objects[%d]: bad 'rotation'", index);
  if (!vec3_of(obj.get("scale"), scale)) return set_error(FR_EPARSE, "objects[%d]: bad 'scale'", index);
  uint32_t mat = FR_LAMBERTIAN;
  V3 color{0.0f, 0.0f, 0.0f};
  float fuzz = 0.0f;
  int rc = material_of(obj, mat, color, fuzz, index);
  if (rc) return rc;

  fr_prim out;
  memset(&out, 0, sizeof(out));
  out.material = mat;
  to_arr(color, out.color);
  out.fuzz = fuzz;
  const Axes ax = quat_axes(q[0], q[1], q[2], q[3]);
  const std::string& m = mesh->text;
  if (m == "sphere") {
    // primitives/sphere.rs:7 RADIUS 0.5, uniformly scaled by scale.x
    out.kind = FR_SPHERE;
    to_arr(pos, out.g);
    out.g[3] = 0.5f * scale.x;
    list.push_back(out);
    return FR_OK;
  }
  if (m == "cube") {
    // primitives/cube.rs:7-38: unit cube, half extent 0.5 per local axis
    const float h[3] = {0.5f * scale.x, 0.5f * scale.y, 0.5f * scale.z};
    int perm[3];
    float sign[3];
    if (signed_permutation(ax, perm, sign)) {
      float hw[3];
      for (int j = 0; j < 3; ++j) hw[perm[j]] = h[j];
      out.kind = FR_AABB;
      out.g[0] = pos.x - hw[0];
      out.g[1] = pos.y - hw[1];
      out.g[2] = pos.z - hw[2];
      out.g[3] = pos.x + hw[0];
      out.g[4] = pos.y + hw[1];
      out.g[5] = pos.z + hw[2];
    } else {
      out.kind = FR_OBB;
      to_arr(pos, out.g);
      to_arr(ax.x, out.g + 3);
      to_arr(ax.y, out.g + 6);
      to_arr(ax.z, out.g + 9);
      out.g[12] = h[0];
      out.g[13] = h[1];
      out.g[14] = h[2];
    }
    list.push_back(out);
    return FR_OK;
  }
  if (m == "triangle") {
    append_mesh(mesh_triangle(), ax, scale, pos, out, list);
    return FR_OK;
  }
  if (m == "circle") {
    append_mesh(mesh_circle(), ax, scale, pos, out, list);
    return FR_OK;
  }
  if (m == "cylinder") {
    append_mesh(mesh_cylinder(30), ax, scale, pos, out, list);
    return FR_OK;
  }
  if (m == "tetrahedron") {
    append_mesh(mesh_tetrahedron(), ax, scale, pos, out, list);
    return FR_OK;
  }
  // "quad" and any other mesh name (basics/scene.rs:93-95 falls back to Quad)
  // primitives/quad.rs:7-12: unit quad in local z = 0 with normal -z. Axis-aligned quads
  // become the reference Plane (orientation = -normal = R*(0,0,1), extent per world
  // axis); any other rotation becomes the quad's two triangles.
  int perm[3];
  float sign[3];
  if (!signed_permutation(ax, perm, sign)) {
    append_mesh(mesh_quad(), ax, scale, pos, out, list);
    return FR_OK;
  }
  const float hl[3] = {0.5f * scale.x, 0.5f * scale.y, 0.0f};
  float size[3], orient[3] = {0.0f, 0.0f, 0.0f};
  for (int j = 0; j < 3; ++j) size[perm[j]] = hl[j];
  size[perm[2]] = size[perm[2]] + 1e-3f;
  orient[perm[2]] = sign[2];
  out.kind = FR_PLANE;
  to_arr(pos, out.g);
  out.g[3] = orient[0];
  out.g[4] = orient[1];
  out.g[5] = orient[2];
  out.g[6] = size[0];
  out.g[7] = size[1];
  out.g[8] = size[2];
  list.push_back(out);
  return FR_OK;
}

}  // namespace
}  // namespace fr

using namespace fr;

extern "C" {

const char* fr_last_error(void) { return g_last_error.c_str(); }

int fr_abi_version(void) { return FR_ABI_VERSION; }

int fr_camera_init(fr_camera* cam, uint32_t width, uint32_t height) {
  if (!cam || width == 0 || height == 0) return set_error(FR_EARG, "fr_camera_init: bad arguments");
  // camera.rs:25-30: look_from (0,0,1), look_at 0, v_up +Y, v_fov 60, aperture 0.1
  const float from[3] = {0.0f, 0.0f, 1.0f}, at[3] = {0.0f, 0.0f, 0.0f}, vup[3] = {0.0f, 1.0f, 0.0f};
  return fr_camera_look(cam, from, at, vup, 60.0f, 0.1f, width, height);
}

int fr_camera_look(fr_camera* cam, const float from[3], const float at[3], const float vup[3], float vfov_deg,
                   float aperture, uint32_t width, uint32_t height) {
  if (!cam || !from || !at || !vup || width == 0 || height == 0)
    return set_error(FR_EARG, "fr_camera_look: bad arguments");
  memset(cam, 0, sizeof(*cam));
  cam->aspect = static_cast<float>(width) / static_cast<float>(height);
  camera_basis(cam, from_arr(from), from_arr(at), from_arr(vup), vfov_deg, aperture);
  cam->focus_dist = 2.0f;  // camera.rs:56 (stored, never used)
  cam->radius = 5.0f;      // camera.rs:57
  cam->rotation = 0.0f;    // camera.rs:58
  return FR_OK;
}

// camera.rs:97-122
int fr_camera_orbit(fr_camera* cam, const float delta[3]) {
  if (!cam || !delta) return set_error(FR_EARG, "fr_camera_orbit: bad arguments");
  cam->rotation += delta[0];
  cam->radius += delta[2];
  cam->position[0] = cam->radius * cosf(cam->rotation);
  cam->position[1] += delta[1];
  cam->position[2] = cam->radius * sinf(cam->rotation);
  const V3 pos = from_arr(cam->position);
  camera_basis(cam, pos, mk(0, 0, 0), mk(0, 1, 0), 60.0f, 0.1f);
  return FR_OK;
}

// camera.rs:74-95
int fr_camera_translate(fr_camera* cam, const float delta[3]) {
  if (!cam || !delta) return set_error(FR_EARG, "fr_camera_translate: bad arguments");
  const V3 pos = add(from_arr(cam->position), from_arr(delta));
  camera_basis(cam, pos, mk(0, 0, -1), mk(0, 1, 0), 60.0f, 0.1f);
  return FR_OK;
}

// tracer.rs:30-50, key bits 00EQADWS
int fr_update_delta(uint8_t keys, float dt, float out[3]) {
  if (!out) return set_error(FR_EARG, "fr_update_delta: null output");
  V3 d = mk(0, 0, 0);
  if ((keys & 0x20) == 0x20) d = add(d, scl(dt, mk(0.0f, -1.0f, 0.0f)));
  if ((keys & 0x10) == 0x10) d = add(d, scl(dt, mk(0.0f, 1.0f, 0.0f)));
  if ((keys & 0x08) == 0x08) d = add(d, scl(dt, mk(1.0f, 0.0f, 0.0f)));
  if ((keys & 0x04) == 0x04) d = add(d, scl(dt, mk(-1.0f, 0.0f, 0.0f)));
  if ((keys & 0x02) == 0x02) d = add(d, scl(dt, mk(0.0f, 0.0f, -1.0f)));
  if ((keys & 0x01) == 0x01) d = add(d, scl(dt, mk(0.0f, 0.0f, 1.0f)));
  to_arr(d, out);
  return FR_OK;
}

int fr_scene_create(const fr_prim* prims, uint32_t n, fr_scene** out) {
  if (!out || (n && !prims)) return set_error(FR_EARG, "fr_scene_create: bad arguments");
  for (uint32_t i = 0; i < n; ++i)
    if (prims[i].kind > FR_TRIANGLE) return set_error(FR_EARG, "fr_scene_create: prims[%u] has unknown kind %u", i, prims[i].kind);
  fr_scene* s = new (std::nothrow) fr_scene();
  if (!s) return set_error(FR_ENOMEM, "fr_scene_create: out of memory");
  s->prims.assign(prims, prims + n);
  *out = s;
  return FR_OK;
}

int fr_scene_builtin(int which, uint32_t width, uint32_t height, fr_scene** out, fr_camera* cam_out) {
  if (!out) return set_error(FR_EARG, "fr_scene_builtin: null output");
  std::vector<fr_prim> prims;
  switch (which) {
    case 0: prims = simple_scene(); break;
    case 1: prims = plane_scene(); break;
    case 2: prims = objects_scene(); break;
    case 3:
      // the state the interactive frontend puts objects[0] in (frontend/macroquad.rs:12-13,66-67)
      prims = simple_scene();
      prims[0].g[0] = -1.0f, prims[0].g[1] = 0.0f, prims[0].g[2] = 0.0f;
      prims[0].g[3] = -1.0f, prims[0].g[4] = 0.0f, prims[0].g[5] = 0.0f;
      break;
    default: return set_error(FR_EARG, "fr_scene_builtin: unknown scene %d", which);
  }
  if (cam_out) {
    int rc = fr_camera_init(cam_out, width, height);
    if (rc) return rc;
  }
  return fr_scene_create(prims.data(), static_cast<uint32_t>(prims.size()), out);
}

int fr_scene_from_json(const char* text, size_t len, uint32_t width, uint32_t height, fr_scene** out,
                       fr_camera* cam_out) {
  if (!text || !out || width == 0 || height == 0) return set_error(FR_EARG, "fr_scene_from_json: bad arguments");
  json::Value root;
  std::string err;
  if (!json::parse(text, len, root, err)) return set_error(FR_EPARSE, "%s", err.c_str());
  if (root.type != json::Value::Object) return set_error(FR_EPARSE, "scene root is not an object");
  // SceneData requires camera, lights and objects (basics/scene_loader.rs:9-14)
  const json::Value* cam = root.get("camera");
  const json::Value* lights = root.get("lights");
  const json::Value* objects = root.get("objects");
  if (!cam || cam->type != json::Value::Object) return set_error(FR_EPARSE, "missing object field 'camera'");
  if (!lights || lights->type != json::Value::Array) return set_error(FR_EPARSE, "missing array field 'lights'");
  if (!objects || objects->type != json::Value::Array) return set_error(FR_EPARSE, "missing array field 'objects'");
  V3 cpos;
  float cq[4], fov;
  if (!vec3_of(cam->get("position"), cpos) || !quat_of(cam->get("rotation"), cq) || !num_f32(cam->get("fov"), fov))
    return set_error(FR_EPARSE, "camera needs position{x,y,z}, rotation{x,y,z,w}, fov");
  std::vector<fr_prim> prims;
  prims.reserve(objects->items.size());
  for (size_t i = 0; i < objects->items.size(); ++i) {
    int rc = map_object(objects->items[i], static_cast<int>(i), prims);
    if (rc) return rc;
  }
  if (cam_out) {
    // JSON camera -> tracer camera: look along the rotated +z axis
    const Axes ax = quat_axes(cq[0], cq[1], cq[2], cq[3]);
    const V3 at = add(cpos, ax.z);
    float f[3], a[3], u[3];
    to_arr(cpos, f);
    to_arr(at, a);
    to_arr(ax.y, u);
    int rc = fr_camera_look(cam_out, f, a, u, fov, 0.1f, width, height);
    if (rc) return rc;
  }
  return fr_scene_create(prims.data(), static_cast<uint32_t>(prims.size()), out);
}

void fr_scene_free(fr_scene* s) {
  if (!s) return;
  release_device_copies(s);
  delete s;
}

uint32_t fr_scene_count(const fr_scene* s) { return s ? static_cast<uint32_t>(s->prims.size()) : 0u; }

int fr_scene_get_prims(const fr_scene* s, fr_prim* out, uint32_t n) {
  if (!s || (n && !out)) return set_error(FR_EARG, "fr_scene_get_prims: bad arguments");
  if (n > s->prims.size()) return set_error(FR_EARG, "fr_scene_get_prims: n > count");
  memcpy(out, s->prims.data(), n * sizeof(fr_prim));
  return FR_OK;
}

// Hitable::translate / rotate (hitable.rs:12-13): only Plane overrides them
// (plane.rs:62-68: position = v, orientation = v); every other shape ignores them.
int fr_scene_translate(fr_scene* s, uint32_t i, const float v[3]) {
  if (!s || !v || i >= s->prims.size()) return set_error(FR_EARG, "fr_scene_translate: bad arguments");
  if (s->prims[i].kind == FR_PLANE) {
    std::lock_guard<std::mutex> g(s->mu);
    memcpy(s->prims[i].g, v, 3 * sizeof(float));
    ++s->version;
  }
  return FR_OK;
}

int fr_scene_rotate(fr_scene* s, uint32_t i, const float v[3]) {
  if (!s || !v || i >= s->prims.size()) return set_error(FR_EARG, "fr_scene_rotate: bad arguments");
  if (s->prims[i].kind == FR_PLANE) {
    std::lock_guard<std::mutex> g(s->mu);
    memcpy(s->prims[i].g + 3, v, 3 * sizeof(float));
    ++s->version;
  }
  return FR_OK;
}

}  // extern "C"
