"""Oracle-side scene construction (TEST INFRASTRUCTURE ONLY).

An independent numpy-float32 restatement of
  * the reference's built-in object lists (cpu_ray_tracer/scenes.rs:6-156) and
    the frontend's plane state (frontend/macroquad.rs:12-13,66-67), and
  * the build's scenes/*.json -> tracer-primitive mapping, which
    reads the serde structs of basics/scene_loader.rs:9-66 and the mesh/material
    dispatch of basics/scene.rs:59-98.

Tests compare the product loader's primitive list (fr_scene_get_prims) with this
one field by field, then render each with its own path. Nothing here is imported
by the product.
"""
from __future__ import annotations

import json
import math

import numpy as np

F = np.float32

SPHERE, PLANE, AABB, OBB, STUB, TRIANGLE = 0, 1, 2, 3, 4, 5
LAMBERTIAN, METAL, DIELECTRIC, LIGHT = 0, 1, 2, 3

# color_utils.rs:101-109 (CP0)
CP0 = [(0.263, 0.208, 0.655), (1.000, 0.498, 0.243), (1.000, 0.965, 0.914), (0.502, 0.769, 0.914)]


def prim(kind, material=0, color=(0.0, 0.0, 0.0), fuzz=0.0, g=()):
    """A primitive record: dict with float32 fields (mirrors or_prim / fr_prim)."""
    gg = np.zeros(16, dtype=F)
    gg[: len(g)] = np.asarray(g, dtype=F)
    return {"kind": int(kind), "material": int(material), "color": np.asarray(color, dtype=F),
            "fuzz": F(fuzz), "g": gg}


def sphere(center, radius, material, color, fuzz):
    return prim(SPHERE, material, color, fuzz, list(center) + [radius])


def plane(position, orientation, size, material, color, fuzz):
    return prim(PLANE, material, color, fuzz, list(position) + list(orientation) + list(size))


def _sqrt3(v):
    return [F(np.sqrt(F(x))) for x in v]


def simple_scene():
    """scenes.rs:6-39"""
    five = [F(5.0) * F(1.0)] * 3
    return [
        plane((-1.0, 0.0, 0.0), (0.0, 0.0, 0.0), five, 1, (1.0, 0.3, 0.3), 0.05),
        sphere((-0.5, 0.0, 0.0), 0.5, 0, (0.0, 0.66, 0.13), 0.0),
        sphere((0.5, 0.0, 0.0), 0.5, 0, (0.7, 0.43, 0.0), 0.0),
        sphere((0.0, -1000.5, 0.0), 1000.0, 0, (0.3, 0.3, 0.3), 1.0),
    ]


def plane_scene():
    """scenes.rs:41-108 (the one uncommented plane)"""
    return [plane((-1.0, 0.0, 0.0), (0.0, 0.0, 0.0), [F(100.0)] * 3, 1, (0.1, 0.9, 0.1), 0.0)]


def objects_scene():
    """scenes.rs:110-156"""
    return [
        sphere((0.0, 0.0, -1.0), 0.5, 0, (0.5, 0.1, 0.1), 0.0),
        sphere((1.0, 0.0, -1.0), 0.5, 1, (0.9, 0.9, 0.9), 0.2),
        sphere((1.0, 0.0, -3.0), 0.5, 1, (1.0, 1.0, 1.0), 1.0),
        sphere((-1.0, -0.0, -1.0), 0.5, 2, _sqrt3(_sqrt3(_sqrt3((0.1, 0.5, 0.1)))), 0.2),
        sphere((0.0, 0.0, 1.0), 0.5, 2, _sqrt3(_sqrt3(_sqrt3((0.5, 0.5, 0.3)))), 0.2),
        sphere((0.0, -100.5, -1.0), 100.0, 0, (0.1, 0.3, 0.9), 0.0),
    ]


def frontend_scene():
    """simple scene with objects[0] translated/rotated as the macroquad frontend does"""
    s = simple_scene()
    s[0]["g"][0:3] = np.asarray((-1.0, 0.0, 0.0), dtype=F)
    s[0]["g"][3:6] = np.asarray((-1.0, 0.0, 0.0), dtype=F)
    return s


BUILTIN = {0: simple_scene, 1: plane_scene, 2: objects_scene, 3: frontend_scene}


# ---- JSON mapping -------------------------------------------

def quat_axes(x, y, z, w):
    """glam Mat3::from_quat columns in f32 (the TRS matrix of primitives/primitive.rs:65-69)."""
    x, y, z, w = F(x), F(y), F(z), F(w)
    x2, y2, z2 = x + x, y + y, z + z
    xx, xy, xz = x * x2, x * y2, x * z2
    yy, yz, zz = y * y2, y * z2, z * z2
    wx, wy, wz = w * x2, w * y2, w * z2
    one = F(1.0)
    ax = [one - (yy + zz), xy + wz, xz - wy]
    ay = [xy - wz, one - (xx + zz), yz + wx]
    az = [xz + wy, yz - wx, one - (xx + yy)]
    return ax, ay, az


def _snap(v):
    a = abs(float(v))
    if a < 1e-5:
        return 0.0
    if abs(a - 1.0) < 1e-5:
        return 1.0 if v > 0 else -1.0
    return None


def signed_permutation(axes):
    """[(world axis, sign) for each local axis] if the rotation is a signed permutation."""
    out, used = [], set()
    for col in axes:
        s = [_snap(c) for c in col]
        if any(c is None for c in s):
            return None
        nz = [i for i, c in enumerate(s) if c != 0.0]
        if len(nz) != 1 or nz[0] in used:
            return None
        used.add(nz[0])
        out.append((nz[0], s[nz[0]]))
    return out


def _f32(text_or_num):
    return F(float(text_or_num))


def _v3(d):
    return [_f32(d["x"]), _f32(d["y"]), _f32(d["z"])]


def _q(d):
    return [_f32(d["x"]), _f32(d["y"]), _f32(d["z"]), _f32(d["w"])]


PALETTE_INDEX = {"EqualizerMaterial": 1, "WaveMaterial": 2, "Texture": 3, "UnlitColorMaterial": 3}
RT_MATERIALS = {"lambertian": LAMBERTIAN, "metal": METAL, "dielectric": DIELECTRIC, "light": LIGHT}


class MappingError(ValueError):
    pass


# ---- meshes as triangle lists (primitives/*.rs vertex/index tables) ----

def _angle(i, n):
    """`i as f32 * 2.0 * PI / n as f32` (circle.rs:67, cylinder.rs:76) in f32."""
    return ((F(i) * F(2.0)) * F(3.14159265358979323846)) / F(n)


def _cos(a):
    return F(math.cos(float(a)))


def _sin(a):
    return F(math.sin(float(a)))


def mesh_triangle():  # triangle.rs:6-13
    return [(0.0, 0.5, 0.0), (-0.5, -0.5, 0.0), (0.5, -0.5, 0.0)], [0, 1, 2]


def mesh_quad():  # quad.rs:7-17
    return [(-0.5, -0.5, 0.0), (0.5, -0.5, 0.0), (0.5, 0.5, 0.0), (-0.5, 0.5, 0.0)], [0, 1, 2, 2, 3, 0]


def mesh_tetrahedron():  # tetrahedron.rs:13-32
    X = 1.0
    v = [(X, X, -X), (X, -X, X), (-X, X, X), (-X, X, X), (-X, -X, -X), (X, X, -X),
         (-X, X, X), (X, -X, X), (-X, -X, -X), (X, X, -X), (-X, -X, -X), (X, -X, X)]
    return v, list(range(12))


def mesh_circle(n=36):  # circle.rs:64-107
    v = [(F(0.5) * _cos(_angle(k, n)), F(0.5) * _sin(_angle(k, n)), 0.0) for k in range(n)] + [(0.0, 0.0, 0.0)]
    idx = []
    for k in range(n):
        idx += [k, (k + 1) % n, n]
    return v, idx


def mesh_cylinder(n=30):  # cylinder.rs:72-174, sector_count 30 (basics/scene.rs:90)
    v = []
    for y in (0.5, -0.5):
        v += [(F(0.5) * _cos(_angle(k, n)), y, F(0.5) * _sin(_angle(k, n))) for k in range(n)]
        v.append((0.0, y, 0.0))
    for y in (0.5, -0.5):
        v += [(F(0.5) * _cos(_angle(k, n)), y, F(0.5) * _sin(_angle(k, n))) for k in range(n)]
    idx = []
    for k in range(n):
        idx += [k, (k + 1) % n, n]
    off = n + 1
    for k in range(n):
        idx += [(k + 1) % n + off, k + off, n + off]
    side = 2 * (n + 1)
    for k in range(n):
        idx += [(k + 1) % n + side, k + side, (k + 1) % n + side + n]
        idx += [k + side + n, (k + 1) % n + side + n, k + side]
    return v, idx


def to_world(axes, scale, pos, l):
    """w = ((ax.x (s.x l.x) + ax.y (s.y l.y)) + ax.z (s.z l.z)) + pos, f32 per component."""
    sx, sy, sz = scale[0] * F(l[0]), scale[1] * F(l[1]), scale[2] * F(l[2])
    ax, ay, az = axes
    return [((ax[i] * sx + ay[i] * sy) + az[i] * sz) + pos[i] for i in range(3)]


def mesh_prims(mesh, axes, scale, pos, material, color, fuzz):
    verts, idx = mesh
    w = [to_world(axes, scale, pos, v) for v in verts]
    return [prim(TRIANGLE, material, color, fuzz, w[idx[t]] + w[idx[t + 1]] + w[idx[t + 2]])
            for t in range(0, len(idx) - 2, 3)]


MESHES = {"triangle": mesh_triangle, "circle": mesh_circle, "cylinder": mesh_cylinder,
          "tetrahedron": mesh_tetrahedron}


def map_object(o):
    """One JSON object -> its list of tracer primitives."""
    mesh, mat_name = o["mesh"], o["material"]
    pos, q, scale = _v3(o["position"]), _q(o["rotation"]), _v3(o["scale"])
    if mat_name == "DiffuseTexture":
        raise MappingError("DiffuseTexture is todo!() in basics/scene.rs:74")
    pal = PALETTE_INDEX.get(mat_name, 0)
    material, color, fuzz = LAMBERTIAN, [F(c) for c in CP0[pal]], F(0.0)
    rt = o.get("rt")
    if rt is not None:
        if "material" in rt:
            material = RT_MATERIALS[rt["material"]]
        if "color" in rt:
            color = [_f32(c) for c in rt["color"]]
        if "fuzz" in rt:
            fuzz = _f32(rt["fuzz"])
    axes = quat_axes(*q)
    half = F(0.5)
    if mesh == "sphere":
        return [prim(SPHERE, material, color, fuzz, pos + [half * scale[0]])]
    if mesh == "cube":
        h = [half * s for s in scale]
        perm = signed_permutation(axes)
        if perm is not None:
            hw = [F(0.0)] * 3
            for j, (i, _) in enumerate(perm):
                hw[i] = h[j]
            mn = [pos[i] - hw[i] for i in range(3)]
            mx = [pos[i] + hw[i] for i in range(3)]
            return [prim(AABB, material, color, fuzz, mn + mx)]
        g = pos + list(axes[0]) + list(axes[1]) + list(axes[2]) + h
        return [prim(OBB, material, color, fuzz, g)]
    if mesh in MESHES:
        return mesh_prims(MESHES[mesh](), axes, scale, pos, material, color, fuzz)
    # "quad" and any unknown mesh (basics/scene.rs:93-95 falls back to Quad)
    perm = signed_permutation(axes)
    if perm is None:
        return mesh_prims(mesh_quad(), axes, scale, pos, material, color, fuzz)
    hl = [half * scale[0], half * scale[1], F(0.0)]
    size, orient = [F(0.0)] * 3, [F(0.0)] * 3
    for j, (i, _) in enumerate(perm):
        size[i] = hl[j]
    iz, sz = perm[2]
    size[iz] = size[iz] + F(1e-3)
    orient[iz] = F(sz)
    return [prim(PLANE, material, color, fuzz, pos + orient + size)]


def camera_of(scene_json):
    """JSON camera -> (from, at, vup, fov): look along the rotated +z axis."""
    cam = scene_json["camera"]
    pos, q = _v3(cam["position"]), _q(cam["rotation"])
    axes = quat_axes(*q)
    at = [pos[i] + axes[2][i] for i in range(3)]
    return pos, at, list(axes[1]), _f32(cam["fov"])


def load_json(text):
    """scene JSON text -> (prims, (from, at, vup, fov))"""
    d = json.loads(text)
    for key in ("camera", "lights", "objects"):
        if key not in d:
            raise MappingError(f"missing field {key!r}")
    return [p for o in d["objects"] for p in map_object(o)], camera_of(d)
