"""Host-side product logic against the oracle's independent restatement (no GPU):
the scenes/*.json -> primitive mapping, the built-in scenes, the camera, the
update() key handling, and the scene generator."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import oracle_py as O
from oracle import scene_ref as S

SCENES_OK = ["scene_01", "scene_02", "scene_03", "scene_04", "scene_05", "scene_06", "scene_07", "scene_08",
             "scene_09"]
REF_SCENES = "/root/reference/scenes"


def _same(prims_c, prims_ref):
    assert len(prims_c) == len(prims_ref)
    for p, q in zip(prims_c, prims_ref):
        assert p.kind == q["kind"] and p.material == q["material"]
        assert np.array_equal(np.array(p.color[:], dtype=np.float32).view(np.uint32), q["color"].view(np.uint32))
        assert np.float32(p.fuzz) == q["fuzz"]
        assert np.array_equal(np.array(p.g[:], dtype=np.float32).view(np.uint32), q["g"].view(np.uint32))


@pytest.mark.parametrize("name", SCENES_OK)
@pytest.mark.parametrize("wh", [(64, 36), (1920, 1080), (31, 17)])
def test_json_scene_matches_oracle(fr, name, wh):
    text = open(fr.scene_path(name)).read()
    sc = fr.Scene.from_json(text, *wh)
    prims, (frm, at, vup, fov) = S.load_json(text)
    _same(sc.prims(), prims)
    cam = O.camera_look(frm, at, vup, fov, 0.1, *wh)
    assert np.array_equal(sc.camera.to_array().view(np.uint32), O.camera_to_array(cam).view(np.uint32))


def test_scene08_slabs(fr):
    sc = fr.Scene.from_file(fr.scene_path("scene_08"), 1920, 1080)
    pr = sc.prims()
    assert [p.kind for p in pr] == [fr.FR_AABB] * 6
    # cube 2 (rotated 90 deg about z, scale 0.1 x 60 x 70) is the floor slab x in [0,60], y = -30 +- 0.05
    assert list(pr[2].g[:6]) == [0.0, np.float32(-30.05), -35.0, 60.0, np.float32(-29.95), 35.0]


@pytest.mark.skipif(not os.path.isdir(REF_SCENES), reason="reference checkout not present (GPU box)")
def test_bundled_scenes_parse_like_the_reference_files(fr):
    for name in SCENES_OK:
        a = json.load(open(os.path.join(REF_SCENES, f"{name}.json")))
        b = json.load(open(fr.scene_path(name)))
        assert a == b


@pytest.mark.parametrize("which", [0, 1, 2, 3])
def test_builtin_scenes(fr, which):
    sc = fr.Scene.builtin(which, 64, 48)
    _same(sc.prims(), S.BUILTIN[which]())
    assert np.array_equal(sc.camera.to_array(), O.camera_to_array(O.camera_new(64, 48)))


def test_translate_rotate_only_move_planes(fr):
    sc = fr.Scene.builtin(0, 8, 8)
    sc.translate(0, (-1.0, 0.0, 0.0))
    sc.rotate(0, (-1.0, 0.0, 0.0))
    sc.translate(1, (9.0, 9.0, 9.0))  # Sphere keeps the trait's no-op (hitable.rs:12)
    _same(sc.prims(), S.BUILTIN[3]())


@pytest.mark.parametrize("name,kinds", [
    ("scene_02", {1: 1, 5: 36 + 120}),        # quad (Plane) + circle (36) + cylinder (30 sectors: 120)
    ("scene_06", {1: 1, 5: 12 * 120}),        # quad + 12 cylinders
    ("scene_09", {5: 4})])                    # tetrahedron
def test_meshes_become_triangle_lists(fr, name, kinds):
    """basics/scene.rs:81-95 meshes: circle/cylinder/tetrahedron/triangle -> triangle lists
    (primitives/*.rs vertex and index tables)."""
    import collections
    sc = fr.Scene.from_file(fr.scene_path(name), 64, 36)
    assert dict(collections.Counter(p.kind for p in sc.prims())) == kinds


def _one_object(mesh, rot=(0.0, 0.0, 0.0, 1.0), scale=(1.0, 1.0, 1.0)):
    return json.dumps({"camera": {"position": {"x": 0, "y": 0, "z": -5}, "rotation": {"x": 0, "y": 0, "z": 0, "w": 1},
                                  "fov": 60}, "lights": [],
                       "objects": [{"mesh": mesh, "material": "DiffuseColorMaterial",
                                    "position": {"x": 0.25, "y": -0.5, "z": 1.0},
                                    "rotation": dict(zip("xyzw", rot)), "scale": dict(zip("xyz", scale))}]})


@pytest.mark.parametrize("mesh,rot,n", [
    ("triangle", (0.0, 0.0, 0.0, 1.0), 1),
    ("triangle", (0.1913417, 0.0, 0.0, 0.98078528), 1),
    ("tetrahedron", (0.46193978, 0.1913417, 0.1913417, 0.84462326), 4),
    ("circle", (0.0, 0.70710677, 0.0, 0.70710677), 36),
    ("cylinder", (0.3, 0.1, -0.2, 0.9273618), 120),
    ("quad", (0.1913417, 0.0, 0.0, 0.98078528), 2),     # tilted quad: its two triangles
    ("pyramid", (0.1913417, 0.0, 0.0, 0.98078528), 2),  # unknown mesh -> Quad (basics/scene.rs:93-95)
    ("pyramid", (0.0, 0.0, 0.0, 1.0), 1)])              # ... axis-aligned: the Plane
def test_mesh_vertices_match_oracle(fr, mesh, rot, n):
    text = _one_object(mesh, rot, (2.0, 0.5, 3.0))
    sc = fr.Scene.from_json(text, 16, 16)
    prims = S.load_json(text)[0]
    assert len(prims) == n
    _same(sc.prims(), prims)


def test_triangle_mesh_vertex_positions():
    # triangle.rs:6-13 under identity rotation, scale (2, 0.5, 3), position (0.25, -0.5, 1)
    p = S.load_json(_one_object("triangle", scale=(2.0, 0.5, 3.0)))[0][0]
    assert list(p["g"][:9]) == [0.25, -0.25, 1.0, -0.75, -0.75, 1.0, 1.25, -0.75, 1.0]


@pytest.mark.parametrize("text", [b"", b"{", b"[1,2]", b'{"camera": {}}', b'{"camera":{"position":{"x":0,"y":0,"z":0},'
                                  b'"rotation":{"x":0,"y":0,"z":0,"w":1},"fov":60},"lights":[],"objects":[{}]}',
                                  b'{"a": 1} trailing'])
def test_malformed_json_is_a_parse_error(fr, text):
    with pytest.raises(fr.ForMaError) as e:
        fr.Scene.from_json(text, 8, 8)
    assert e.value.code == fr.FR_EPARSE


def test_rt_material_extension(fr):
    d = json.loads(open(fr.scene_path("scene_08")).read())
    d["objects"][2]["rt"] = {"material": "metal", "color": [0.9, 0.8, 0.7], "fuzz": 0.1}
    d["objects"][3]["rt"] = {"material": "dielectric"}
    d["objects"].append({"mesh": "sphere", "material": "x", "position": {"x": 10, "y": 0, "z": 0},
                         "rotation": {"x": 0, "y": 0, "z": 0, "w": 1}, "scale": {"x": 4, "y": 4, "z": 4},
                         "rt": {"material": "light"}})
    text = json.dumps(d)
    sc = fr.Scene.from_json(text, 16, 16)
    _same(sc.prims(), S.load_json(text)[0])
    assert [p.material for p in sc.prims()] == [0, 0, 1, 2, 0, 0, 3]


def test_bad_args_are_errors(fr):
    with pytest.raises(fr.ForMaError):
        fr.Scene.from_json(b"{}", 0, 8)
    with pytest.raises(fr.ForMaError):
        fr.Scene.builtin(9, 8, 8)
    bad = fr.FrPrim()
    bad.kind = 99
    with pytest.raises(fr.ForMaError):
        fr.Scene.from_prims([bad])


@pytest.mark.parametrize("delta", [(0.0, 0.0, 0.0), (0.3, -0.2, 0.5), (-1.0, 1.0, -0.25)])
def test_camera_orbit_and_translate_match_oracle(fr, delta):
    a, b = fr.camera_new(320, 200), O.camera_new(320, 200)
    for _ in range(3):
        fr.camera_orbit(a, delta)
        O.camera_orbit(b, delta)
        assert np.array_equal(a.to_array().view(np.uint32), O.camera_to_array(b).view(np.uint32))
    fr.camera_translate(a, delta)
    O.camera_translate(b, delta)
    assert np.array_equal(a.to_array().view(np.uint32), O.camera_to_array(b).view(np.uint32))


def test_zero_orbit_moves_camera_to_radius_5(fr):
    # tracer.rs:52 orbits every frame: from (0,0,1) to (5 cos 0, 0, 5 sin 0)
    c = fr.camera_orbit(fr.camera_new(64, 64), (0.0, 0.0, 0.0))
    assert list(c.position) == [5.0, 0.0, 0.0]


def test_update_key_bitmask(fr):
    import ctypes as C
    out = (C.c_float * 3)()
    fr.check(fr.lib().fr_update_delta(0b101011, 0.5, out))  # E, A, W, S (tracer.rs:33-50)
    assert list(out) == [0.5, -0.5, 0.0]
    fr.check(fr.lib().fr_update_delta(0b010100, 2.0, out))  # Q, D
    assert list(out) == [-2.0, 2.0, 0.0]


def test_generator_matches_reference_generator_output():
    from tools.gen_scene import dumps, generator_scene
    pin = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "generator_100_cubes.json")))
    data = dumps(generator_scene(100, "cube")).encode()
    assert len(data) == pin["bytes"] and hashlib.sha256(data).hexdigest() == pin["sha256"]


def test_generated_scenes_load(fr):
    from tools.gen_scene import dumps, generator_scene
    text = dumps(generator_scene(100, "cube"))
    sc = fr.Scene.from_json(text, 32, 32)
    assert len(sc) == 100 and {p.kind for p in sc.prims()} == {fr.FR_OBB}
    _same(sc.prims(), S.load_json(text)[0])
    text = dumps(generator_scene(10000, "sphere"))
    sc = fr.Scene.from_json(text, 32, 32)
    assert len(sc) == 10000 and sc.prims()[9999].g[3] == 2.5
