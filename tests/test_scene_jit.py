"""The scene-specialised trace kernel (FR_FLAG_SCENE_JIT, fo-rma_amd/csrc/jit.cpp).

trace_kernel.h is compiled again at run time by hiprtc with the scene's primitive records
as constants; only the closest-hit list walk changes (an unrolled sequence of the same
tests, in list order), so every image must equal the oracle's bit for bit, as the
compiled-in kernels' do (test_gpu_parity.py). The CPU tests check that the embedded
sources compile for gfx950 without a device."""
import ctypes as C
import os
import struct

import numpy as np
import pytest

from oracle import oracle_py as O
from oracle import scene_ref as S
from tests.golden import make_golden as G
from tests.test_gpu_parity import GOLDEN, _product_scene, assert_parity, random_scene

JIT_MAX = 64  # jit.h kJitMaxPrims


def _box_records(prims):
    """64-B device records (render.hip upload_scene) of axis-aligned boxes."""
    words = []
    for p in prims:
        g = list(p.g[:6]) if hasattr(p, "g") else p
        rec = list(struct.unpack("16I", struct.pack("16f", g[0], g[1], g[2], 0, g[3], g[4], g[5], 0, *([0.0] * 8))))
        rec[15] = 2  # FR_AABB in g3.w
        words += rec
    return (C.c_uint32 * len(words))(*words), len(words) // 16


def _probe(fr, recs, n, targs=None):
    nb, ms = C.c_size_t(0), C.c_double(0.0)
    ta = None if targs is None else (C.c_int * 8)(*targs)
    rc = fr.lib().fr_selftest_jit(b"gfx950", recs, n, ta, C.byref(nb), C.byref(ms))
    return rc, nb.value, ms.value


def test_scene_kernel_compiles_for_gfx950_without_a_device(fr):
    sc = fr.Scene.from_file(fr.scene_path("scene_08"), 64, 36)
    recs, n = _box_records(sc.prims())
    rc, nbytes, ms = _probe(fr, recs, n)
    assert rc == 0, fr.lib().fr_last_error()
    assert n == 6 and nbytes > 4096


def test_scene_kernel_compiles_at_the_unrolled_bound(fr):
    r = np.random.default_rng(5)
    boxes = []
    for _ in range(15):  # kNibbleMaxPrims: the headline specialisation's largest list
        c, h = r.uniform(-3, 3, 3), r.uniform(0.1, 1, 3)
        boxes.append(list(c - h) + list(c + h))
    recs, n = _box_records(boxes)
    rc, nbytes, _ = _probe(fr, recs, n)
    assert rc == 0, fr.lib().fr_last_error()
    assert nbytes > 4096


def test_scene_kernel_probe_rejects_bad_sizes(fr):
    recs, _ = _box_records([[0, 0, 0, 1, 1, 1]])
    assert _probe(fr, recs, 0)[0] == fr.FR_EARG
    assert _probe(fr, recs, JIT_MAX + 1)[0] == fr.FR_EARG


# ---- on the device --------------------------------------------------------------

def _ctx_render(fr, sc, cam, w, h, spp, depth, seed=None, jit="wait", mt=False):
    ctx = fr.RenderContext(0)
    try:
        kw = {} if seed is None else {"seed": seed}
        ctx.render(sc, cam, fr.make_params(w, h, spp, depth, scene_jit=jit, mt_bands=mt, **kw))
        st = ctx.sync()
        mean, u8 = ctx.download(w, h)
        return mean, u8, st, ctx.jit_info()
    finally:
        ctx.close()


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(G.CASES))
def test_scene_jit_golden_cases(gpu, name):
    spec, w, h, spp, depth, seed = G.CASES[name]
    sc = _product_scene(gpu, spec, w, h)
    mean, u8, st, info = _ctx_render(gpu, sc, sc.camera, w, h, spp, depth, seed)
    # list-loop scenes (< 48 primitives: bvh.h kBvhMinPrims) run the scene kernel; > 64 never
    if 1 <= len(sc) < 48:
        assert info["used"], (len(sc), info)
    elif len(sc) > JIT_MAX or len(sc) == 0:
        assert not info["used"], (len(sc), info)
    ref = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    cnt = {"segments": int(ref["counters"][0]), "hits": int(ref["counters"][1])}
    assert_parity(mean, u8, st, ref["mean"], ref["u8"], cnt)
    assert np.array_equal(mean.view(np.uint32), ref["mean"].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(8))
def test_scene_jit_random_scenes_all_kinds_and_materials(gpu, seed):
    """Spheres, planes (stale records), boxes, oriented boxes, triangles, stubs; every
    material (general shading), against the oracle."""
    w, h, spp, depth = 40, 24, 3, 8 if seed < 6 else 12
    prims = random_scene(seed, n=12 + 4 * seed)  # <= 41 primitives: the list loop
    sc = gpu.Scene.from_prims(prims)
    cam, ocam = gpu.camera_new(w, h), O.camera_new(w, h)
    if seed % 2:
        gpu.camera_orbit(cam, (0.4 * seed, 0.1, -2.0))
        O.camera_orbit(ocam, (0.4 * seed, 0.1, -2.0))
    mean, u8, st, info = _ctx_render(gpu, sc, cam, w, h, spp, depth, seed=2000 + seed)
    assert info["used"]
    omean, ou8, ocnt, _ = O.render(prims, ocam, w, h, spp, depth, seed=2000 + seed, threads=8)
    assert_parity(mean, u8, st, omean, ou8, ocnt)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [2, 5])
def test_scene_jit_diffuse_only_scenes(gpu, seed):
    w, h, spp, depth = 40, 24, 4, 8
    prims = random_scene(seed)
    for q in prims:
        if q["material"] in (S.METAL, S.DIELECTRIC):
            q["material"] = S.LIGHT if seed % 2 else S.LAMBERTIAN
    sc = gpu.Scene.from_prims(prims)
    mean, u8, st, info = _ctx_render(gpu, sc, gpu.camera_new(w, h), w, h, spp, depth, seed=300 + seed)
    assert info["used"]
    omean, ou8, ocnt, _ = O.render(prims, O.camera_new(w, h), w, h, spp, depth, seed=300 + seed, threads=8)
    assert_parity(mean, u8, st, omean, ou8, ocnt)


@pytest.mark.gpu
def test_scene_jit_at_and_past_the_size_bound(gpu, monkeypatch):
    """64 primitives compile into the kernel; 65 run the compiled-in kernel. Both match.
    (FR_BVH=0: the list loop, which scenes of 48 or more primitives otherwise leave.)"""
    monkeypatch.setenv("FR_BVH", "0")
    w, h, spp, depth = 32, 20, 2, 8
    for n, expect in ((JIT_MAX, True), (JIT_MAX + 1, False)):
        r = np.random.default_rng(n)
        prims = []
        for i in range(n - 1):
            c = r.uniform(-3, 3, 3) + np.array([0, 0, -6.0])
            prims.append(S.sphere(c, r.uniform(0.1, 0.4), int(i % 4), r.uniform(0.2, 1, 3), 0.2)
                         if i % 2 else S.prim(S.AABB, 0, r.uniform(0.2, 1, 3), 0.0,
                                              list(c - 0.2) + list(c + 0.3)))
        prims.append(S.sphere((0.0, -100.5, -1.0), 100.0, 0, (0.5, 0.5, 0.5), 0.0))
        sc = gpu.Scene.from_prims(prims)
        mean, u8, st, info = _ctx_render(gpu, sc, gpu.camera_new(w, h), w, h, spp, depth, seed=7)
        assert info["used"] == expect
        omean, ou8, ocnt, _ = O.render(prims, O.camera_new(w, h), w, h, spp, depth, seed=7, threads=8)
        assert_parity(mean, u8, st, omean, ou8, ocnt)


@pytest.mark.gpu
def test_scene_jit_follows_scene_edits_and_reuses_modules(gpu):
    """A translated primitive is a new scene kernel (its constants changed); rendering the
    same scene again reuses the loaded module (no compile, no load)."""
    w, h, spp, depth = 40, 24, 3, 8
    sc = gpu.Scene.builtin(0, w, h)
    cam = gpu.camera_new(w, h)
    a = _ctx_render(gpu, sc, cam, w, h, spp, depth, seed=11)
    b = _ctx_render(gpu, sc, cam, w, h, spp, depth, seed=11)
    assert a[3]["used"] and b[3]["used"] and b[3]["ms"] < 50.0 and not b[3]["compiled"]
    assert np.array_equal(a[0].view(np.uint32), b[0].view(np.uint32))
    sc.translate(0, (-1.0, 0.0, 0.0))
    sc.rotate(0, (-1.0, 0.0, 0.0))
    c = _ctx_render(gpu, sc, cam, w, h, spp, depth, seed=11)
    assert c[3]["used"] and not np.array_equal(a[0], c[0])
    omean, ou8, ocnt, _ = O.render(S.BUILTIN[3](), O.camera_new(w, h), w, h, spp, depth, seed=11, threads=8)
    assert_parity(c[0], c[1], c[2], omean, ou8, ocnt)


@pytest.mark.gpu
@pytest.mark.parametrize("which,w,h,sample", [(0, 32, 18, 3), (2, 36, 22, 20)])
def test_scene_jit_save_image_mt_bands(gpu, which, w, h, sample):
    sc = gpu.Scene.builtin(which, w, h)
    cam = gpu.camera_new(w, h)
    mean, u8, st, info = _ctx_render(gpu, sc, cam, w, h, sample, 50, mt=True)
    assert info["used"]
    ref, ref_u8, _, _ = _ctx_render(gpu, sc, cam, w, h, sample, 50, jit=False, mt=True)
    assert np.array_equal(mean.view(np.uint32), ref.view(np.uint32)) and np.array_equal(u8, ref_u8)
    oacc, ou8, _ = O.render_mt(S.BUILTIN[which](), O.camera_new(w, h), w, h, sample, 50, 0x5EED)
    assert np.array_equal(mean.view(np.uint32), oacc.view(np.uint32)) and np.array_equal(u8, ou8)


@pytest.mark.gpu
def test_scene_jit_shards_and_small_grids(gpu, monkeypatch):
    """Row shards stitch to the unsharded frame, and a tiny persistent grid (every wave
    claims many batches) gives the same image, through the scene kernel."""
    w, h, spp, depth = 64, 40, 40, 8
    sc = gpu.Scene.from_file(gpu.scene_path("scene_08"), w, h)
    full, fu8, _ = gpu.render(sc, sc.camera, w, h, spp, depth, scene_jit="wait")
    for k in range(3):
        m, u, _ = gpu.render(sc, sc.camera, w, h, spp, depth, shard_index=k, shard_count=3, scene_jit="wait")
        rows = [y for y in range(h) if (y // 8) % 3 == k]
        assert np.array_equal(m[rows].view(np.uint32), full[rows].view(np.uint32))
    monkeypatch.setenv("FR_MAX_WGS", "1")
    m, u, _ = gpu.render(sc, sc.camera, w, h, spp, depth, scene_jit="wait")
    assert np.array_equal(m.view(np.uint32), full.view(np.uint32)) and np.array_equal(u, fu8)
    prims, (frm, at, vup, fov) = S.load_json(open(gpu.scene_path("scene_08")).read())
    cam = O.camera_look(frm, at, vup, fov, 0.1, w, h)
    omean, ou8, _, _ = O.render(prims, cam, w, h, spp, depth, threads=8)
    assert np.array_equal(full.view(np.uint32), omean.view(np.uint32))


@pytest.mark.gpu
def test_prepare_gets_the_scene_kernel_before_the_first_frame(gpu):
    """fr_ctx_prepare sets a render up without rendering: afterwards the first frame runs
    the scene kernel without compiling or loading it (bench.py's untimed set-up)."""
    w, h, spp, depth = 48, 32, 8, 8
    sc = gpu.Scene.from_file(gpu.scene_path("scene_08"), w, h)
    p = gpu.make_params(w, h, spp, depth, scene_jit="wait")
    ctx = gpu.RenderContext(0)
    try:
        info = ctx.prepare(sc, sc.camera, p)
        assert info["used"]
        ctx.render(sc, sc.camera, p)
        st = ctx.sync()
        after = ctx.jit_info()
        assert after["used"] and not after["compiled"] and after["ms"] < 50.0
        mean, u8 = ctx.download(w, h)
    finally:
        ctx.close()
    ref, ref_u8, ref_st = gpu.render(sc, sc.camera, w, h, spp, depth)
    assert np.array_equal(mean.view(np.uint32), ref.view(np.uint32)) and np.array_equal(u8, ref_u8)
    assert st["segments"] == ref_st["segments"]


# ---- background compile, fallback and the disk cache (jit.cpp) ----------------------

def _fresh_boxes(seed, n=9):
    """A diffuse box scene no other test renders (its scene kernel exists nowhere yet)."""
    r = np.random.default_rng(seed)
    prims = []
    for _ in range(n):
        c, hx = r.uniform(-3, 3, 3) + np.array([0, 0, -7.0]), r.uniform(0.2, 1.2, 3)
        prims.append(S.prim(S.AABB, 0, r.uniform(0.2, 0.9, 3), 0.0, list(c - hx) + list(c + hx)))
    return prims


@pytest.mark.gpu
def test_first_frames_fall_back_bit_identically_while_compiling(gpu, tmp_path, monkeypatch):
    """FR_FLAG_SCENE_JIT without _WAIT never blocks a render on hiprtc: with no code object
    in the process or on disk, the first frame queues the compile and runs the compiled-in
    kernel (state PENDING), bit for bit the image the flag-off render gives; once the
    background compile is done, the next frame runs the scene kernel (USED), same bits."""
    monkeypatch.setenv("FR_JIT_CACHE", str(tmp_path))
    w, h, spp, depth = 48, 32, 6, 8
    prims = _fresh_boxes(9071)
    sc = gpu.Scene.from_prims(prims)
    cam = gpu.camera_new(w, h)
    ref = _ctx_render(gpu, sc, cam, w, h, spp, depth, jit=False)
    ctx = gpu.RenderContext(0)
    try:
        p = gpu.make_params(w, h, spp, depth, scene_jit=True)
        ctx.render(sc, cam, p)
        st1 = ctx.sync()
        first = ctx.download(w, h) + (ctx.jit_info(),)
        assert first[2]["state"] == gpu.FR_JIT_PENDING and not first[2]["used"], first[2]
        assert first[2]["ms"] < 50.0  # the render did not wait for hiprtc
        gpu.jit_wait()
        ctx.render(sc, cam, p)
        st2 = ctx.sync()
        second = ctx.download(w, h) + (ctx.jit_info(),)
        assert second[2]["state"] == gpu.FR_JIT_USED and second[2]["used"], second[2]
    finally:
        ctx.close()
    for mean, u8, st in ((first[0], first[1], st1), (second[0], second[1], st2)):
        assert np.array_equal(mean.view(np.uint32), ref[0].view(np.uint32)) and np.array_equal(u8, ref[1])
        assert (st["segments"], st["hits"], st["scatters"]) == (ref[2]["segments"], ref[2]["hits"], ref[2]["scatters"])
    assert len(list(tmp_path.glob("*.hsaco"))) == 1  # the background compile filled the disk cache
    omean, ou8, ocnt, _ = O.render(prims, O.camera_new(w, h), w, h, spp, depth, threads=8)
    assert_parity(first[0], first[1], st1, omean, ou8, ocnt)


_RENDER_ONCE = """
import json, sys
sys.path.insert(0, {pkg!r}); sys.path.insert(0, {root!r})
import numpy as np
import forma_rt as fr
from tests.test_scene_jit import _fresh_boxes
sc = fr.Scene.from_prims(_fresh_boxes(6113))
cam = fr.camera_new(40, 24)
ctx = fr.RenderContext(0)
ctx.render(sc, cam, fr.make_params(40, 24, 4, 8, scene_jit="wait"))
ctx.sync()
mean, u8 = ctx.download(40, 24)
print(json.dumps(dict(ctx.jit_info(), sha=__import__("hashlib").sha256(mean.tobytes()).hexdigest())))
"""


def _render_in_fresh_process(cache):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = _RENDER_ONCE.format(pkg=os.path.join(root, "fo-rma_amd"), root=root)
    env = dict(os.environ, FR_JIT_CACHE=str(cache))
    out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    import json
    return json.loads(out.stdout.strip().splitlines()[-1])


@pytest.mark.gpu
@pytest.mark.parametrize("damage", ["truncate", "garbage"])
def test_damaged_cache_file_is_rebuilt(gpu, tmp_path, damage):
    """A code object in the disk cache that does not load (truncated by a full disk, or not
    a code object at all) is deleted and compiled again: the render succeeds with the scene
    kernel and the same image, and the cache holds a good file afterwards."""
    a = _render_in_fresh_process(tmp_path)
    assert a["used"] and a["compiled"], a
    (f,) = list(tmp_path.glob("*.hsaco"))
    good = f.read_bytes()
    f.write_bytes(good[: len(good) // 3] if damage == "truncate" else os.urandom(4096))
    b = _render_in_fresh_process(tmp_path)
    assert b["used"] and b["compiled"] and b["sha"] == a["sha"], b
    (f2,) = list(tmp_path.glob("*.hsaco"))
    assert f2.read_bytes() == good
    c = _render_in_fresh_process(tmp_path)  # and a third process loads it without compiling
    assert c["used"] and not c["compiled"] and c["sha"] == a["sha"], c


@pytest.mark.gpu
def test_one_shot_save_image_through_mctx_on_a_cold_cache(gpu, tmp_path):
    """The reference's one caller renders one image once (frontend/macroquad.rs:60,
    save_image(&mut model, 50)). Through fr_mctx at 1920x1080 with the scene kernel asked
    for and no code object anywhere, the frame costs at most 1.5x the compiled-in kernel's
    (it runs the compiled-in kernel while hiprtc works in the background), every image is
    the same bits, and the frame after the compile runs the scene kernel on every shard."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FR_JIT_CACHE=str(tmp_path))
    out = subprocess.run([sys.executable, os.path.join(root, "tools", "jit_cold.py"), "--devices", "0,0"], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    print(r)
    assert r["bit_identical"], r
    assert r["cold_states"] == [2, 2] and r["hot_states"] == [1, 1], r
    assert r["ratio"] <= 1.5, r


_ONE_SHOT = r'''
import json, os, sys, time
sys.path.insert(0, os.path.join(sys.argv[1], "fo-rma_amd"))
import forma_rt as fr
t0 = time.perf_counter()
m = fr.create_model(320, 180, fr.Scene.from_file(fr.scene_path("scene_08"), 320, 180))
if sys.argv[2] == "warm":  # compile the kernel save_image will look up, on this thread
    m.render(m.scene, 8, fr.MAX_DEPTH, m.seed, scene_jit="wait")
mean, u8, st = fr.save_image(m, 8, path=os.path.join(sys.argv[3], "one_shot.png"))
print(json.dumps({"state": m.ctx.jit_state(), "ms": (time.perf_counter() - t0) * 1e3,
                  "sha": __import__("hashlib").sha256(mean.tobytes()).hexdigest()[:16]}))
'''


@pytest.mark.gpu
def test_one_shot_save_image_never_queues_a_compile(gpu, tmp_path):
    """save_image / save_image_mt are one-shot calls (the reference's only caller renders once,
    frontend/macroquad.rs:60): with FR_FLAG_SCENE_JIT_CACHED they use the scene kernel only if
    its code object is cached and otherwise compile nothing, so a process that renders once
    and exits never waits for hiprtc at exit (a queued background compile runs to its end
    there). Cold cache: FR_JIT_MISS, no file written, the compiled-in kernel's bits. Warm
    cache (the same kernel compiled earlier in the process): FR_JIT_USED, the same bits."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cache = tmp_path / "cache"
    cache.mkdir()
    env = dict(os.environ, FR_JIT_CACHE=str(cache))
    env.pop("FR_SCENE_JIT", None)
    res = {}
    for mode in ("cold", "warm"):
        out = subprocess.run([sys.executable, "-c", _ONE_SHOT, root, mode, str(tmp_path)], env=env, capture_output=True,
                             text=True, timeout=300)
        assert out.returncode == 0, out.stderr[-2000:]
        res[mode] = json.loads(out.stdout.strip().splitlines()[-1])
        if mode == "cold":
            assert res[mode]["state"] == gpu.FR_JIT_MISS, res
            assert not list(cache.iterdir()), "a cold one-shot save_image queued a compile"
    assert res["warm"]["state"] == gpu.FR_JIT_USED, res
    assert res["cold"]["sha"] == res["warm"]["sha"], res


_EVICT = r'''
import hashlib, json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "fo-rma_amd"))
import forma_rt as fr
W, H = 1920, 1080
x = fr.Scene.from_file(fr.scene_path("scene_01"), W, H)
y = fr.Scene.from_file(fr.scene_path("scene_08"), 96, 64)
z = fr.Scene.builtin(0, 96, 64)
px = fr.make_params(W, H, 256, 8, scene_jit="wait")
py, pz = (fr.make_params(96, 64, 8, 8, scene_jit="wait", seed=s) for s in (3, 4))
# every code object compiled once (the module bound is 1, so these loads evict each other)
for sc, p in ((x, fr.make_params(32, 16, 1, 8, scene_jit="wait")), (y, py), (z, pz)):
    c = fr.RenderContext(0); c.render(sc, sc.camera, p); c.sync(); c.close()
a, b = fr.RenderContext(0), fr.RenderContext(0)
a.render(x, x.camera, px)          # ~13 passes, alternating two trace streams; no host wait
a.render(y, y.camera, py)          # A's pin moves to y's module: x's is unpinned, still in flight
b.render(z, z.camera, pz)          # loading z's module evicts x's while its passes run
out = {}
for name, c, w, h in (("y", a, 96, 64), ("z", b, 96, 64)):
    st = c.sync(); m, u = c.download(w, h)
    out[name] = {"sha": hashlib.sha256(m.tobytes()).hexdigest(), "used": c.jit_info()["used"], "seg": st["segments"]}
    c.close()
print(json.dumps(out))
'''


@pytest.mark.gpu
def test_module_eviction_waits_for_every_stream(gpu):
    """an evicted scene-kernel module is unloaded only after the last launch on
    every stream it was launched on. With the module bound forced to 1 (FR_JIT_MAX_MODULES),
    a 13-pass frame (traces alternating between the context's two streams) is still running
    when its module is unpinned and then evicted by another context's load; the process must
    finish without a fault, and the frames rendered around the eviction must equal the
    compiled-in kernel's."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FR_JIT_MAX_MODULES="1", FR_SAMPLE_BUFFER_GB="0.5")
    env.pop("FR_SCENE_JIT", None)
    out = subprocess.run([sys.executable, "-c", _EVICT, root], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    r = json.loads(out.stdout.strip().splitlines()[-1])
    import hashlib
    for name, sc, seed in (("y", gpu.Scene.from_file(gpu.scene_path("scene_08"), 96, 64), 3),
                           ("z", gpu.Scene.builtin(0, 96, 64), 4)):
        m, u, st = gpu.render(sc, sc.camera, 96, 64, 8, 8, seed=seed)
        assert r[name]["used"], r
        assert r[name]["sha"] == hashlib.sha256(m.tobytes()).hexdigest() and r[name]["seg"] == st["segments"], r
