"""GPU parity: the gfx950 kernel (through the C ABI) against the oracle.

Bar (BASELINE.json north star): per-channel |mean_gpu - mean_oracle| <= 1e-5.
The kernel is built to match bit for bit, so these tests also require the u8
image and the path counters (segments, hits) to be identical — counters catch a
control-flow divergence before colour does. Full-size (1080p) configs are
checked on a deterministic row subset that the oracle finishes in seconds.
"""
import os

import numpy as np
import pytest

from oracle import oracle_py as O
from oracle import scene_ref as S
from tests.golden import make_golden as G

pytestmark = pytest.mark.gpu
TOL = 1e-5  # north-star tolerance, f32 means per channel
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def assert_parity(mean, u8, st, omean, ou8, ocnt, rows=None):
    if rows is not None:
        mean, u8, omean, ou8 = mean[rows], u8[rows], omean[rows], ou8[rows]
    assert not np.isnan(mean).any()
    err = float(np.max(np.abs(mean - omean))) if mean.size else 0.0
    assert err <= TOL, f"max |d| = {err}"
    assert np.array_equal(u8, ou8), f"u8 differs at {np.argwhere(u8 != ou8)[:5]}"
    if ocnt is not None:
        assert (st["segments"], st["hits"]) == (ocnt["segments"], ocnt["hits"])
        if "scatters" in ocnt:
            assert st["scatters"] == ocnt["scatters"]
    return err


# ---- device arithmetic --------------------------------------------------------

def _edge_floats(rng, n):
    special = np.array([0.0, -0.0, 1.0, -1.0, 1e-45, -1e-45, 1.17549435e-38, 3.4e38, -3.4e38, np.inf, -np.inf,
                        np.nan, 0.5, 2.0, 1e-20, 1e20, 0.001, 1.3], dtype=np.float32)
    bits = rng.integers(0, 2 ** 32, size=n, dtype=np.uint64).astype(np.uint32).view(np.float32)
    normal = rng.standard_normal(n).astype(np.float32) * np.float32(10.0)
    return np.concatenate([special, bits, normal]).astype(np.float32)


def _same_bits(a, b):
    both_nan = np.isnan(a) & np.isnan(b)
    return np.all(both_nan | (a.view(np.uint32) == b.view(np.uint32)))


@pytest.mark.parametrize("op", ["add", "sub", "mul", "div", "sqrt", "recip"])
def test_device_arithmetic_is_ieee_correctly_rounded(gpu, op):
    import ctypes as C
    rng = np.random.default_rng(1)
    a = _edge_floats(rng, 20000)
    b = np.roll(_edge_floats(rng, 20000), 7)
    b = b[: a.size]
    code = {"add": 0, "sub": 1, "mul": 2, "div": 3, "sqrt": 4, "recip": 8}[op]
    out = np.empty_like(a)
    fp = C.POINTER(C.c_float)
    gpu.check(gpu.lib().fr_selftest_ops(0, code, a.ctypes.data_as(fp), b.ctypes.data_as(fp), a.size,
                                        out.ctypes.data_as(fp)))
    with np.errstate(all="ignore"):
        want = {"add": a + b, "sub": a - b, "mul": a * b, "div": a / b, "sqrt": np.sqrt(a),
                "recip": np.float32(1.0) / a}[op]
    assert _same_bits(out, want.astype(np.float32))


def test_recip_nr_exhaustive(gpu):
    """rcp + one FMA Newton step equals the correctly rounded 1.0f / x for every f32 whose
    exponent field is 1..252; the kernel's guard (recip_nr_ok) sends all others, and only
    those, to the IEEE division. All 2^32 bit patterns are checked on the device."""
    import ctypes as C
    bad = np.zeros(256, np.uint64)
    first = np.zeros(256, np.uint32)
    gpu.check(gpu.lib().fr_selftest_recip(0, 0, 1 << 32, bad.ctypes.data_as(C.POINTER(C.c_uint64)),
                                          first.ctypes.data_as(C.POINTER(C.c_uint32))))
    assert not bad[1:253].any(), {e: (int(bad[e]), hex(int(first[e]))) for e in np.nonzero(bad[1:253])[0] + 1}


def test_div_rn_exhaustive(gpu):
    """div_rn (q0 = a y, one FMA residual correction, y = RN(1 / b)) equals the IEEE
    division for all 2^46 operand pairs in [1, 2) x [1, 2), the mantissa space every
    in-range use (jitter, sky parameter, sphere roots) scales to exactly."""
    import ctypes as C
    bad = C.c_uint64(0)
    first = C.c_uint64(0)
    gpu.check(gpu.lib().fr_selftest_div(0, 0, 1 << 23, C.byref(bad), C.byref(first)))
    assert bad.value == 0, (bad.value, hex(first.value >> 23), hex(first.value & 0x7FFFFF))


def test_device_max3_and_min3_match_fmaxf_fminf(gpu):
    """The slab test's v_max3_f32 (tn) and v_min3_f32 (tf) against the host's fmaxf/fminf
    chains, bit for bit, on edge values (NaN, +-0, +-inf, denormals). Slab distances come
    from arithmetic, which only makes quiet NaNs; signalling NaNs (which IEEE-mode v_max /
    v_min quiet and propagate one step) are quieted for the host comparison, and v_max3 /
    v_min3 must equal the chained v_max_f32 / v_min_f32 on them as on everything."""
    import ctypes as C
    rng = np.random.default_rng(12)
    fp = C.POINTER(C.c_float)

    def quiet(a):
        u = a.view(np.uint32).copy()
        snan = ((u & 0x7F800000) == 0x7F800000) & ((u & 0x007FFFFF) != 0)
        u[snan] |= 0x00400000
        return u.view(np.float32)

    def run(op, x, y):
        out = np.empty_like(x)
        gpu.check(gpu.lib().fr_selftest_ops(0, op, x.ctypes.data_as(fp), y.ctypes.data_as(fp), x.size,
                                            out.ctypes.data_as(fp)))
        return out

    x_raw = _edge_floats(rng, 50000)
    y_raw = np.roll(_edge_floats(rng, 50000), 3)[: x_raw.size]
    assert _same_bits(run(11, x_raw, y_raw), run(13, x_raw, y_raw))  # max3 == chained v_max, sNaN included
    assert _same_bits(run(12, x_raw, y_raw), run(17, x_raw, y_raw))  # min3 == chained v_min, sNaN included
    x, y = quiet(x_raw), quiet(y_raw)
    z = np.roll(y, -1)
    for op, f in ((11, np.fmax), (12, np.fmin)):
        out = run(op, x, y)
        want = f(f(x, y), z)
        # fmaxf/fminf leave the sign of equal zeros unspecified; the slab test never depends on it
        zero = (want == 0) & (out == 0)
        assert _same_bits(out[~zero], want[~zero]), op


def test_guarded_recip_and_jitter_division(gpu):
    """The kernel's fast reciprocal with its range guard (op 10) and its jitter division
    div_rn((x + r) , W, RN(1/W)) (op 9) against numpy's IEEE float32 division."""
    import ctypes as C
    rng = np.random.default_rng(11)
    fp = C.POINTER(C.c_float)
    x = _edge_floats(rng, 200000)
    tiny = np.array([1e-38, -1e-38, 2.0 ** -126, -(2.0 ** -126), 2.0 ** -127, 2.0 ** 126, 2.0 ** 127, 3e38, -3e38,
                     0.0, -0.0, 1e-45], dtype=np.float32)
    x = np.concatenate([x, tiny])
    out = np.empty_like(x)
    gpu.check(gpu.lib().fr_selftest_ops(0, 10, x.ctypes.data_as(fp), x.ctypes.data_as(fp), x.size,
                                        out.ctypes.data_as(fp)))
    with np.errstate(all="ignore"):
        assert _same_bits(out, np.float32(1.0) / x)
    for wh in (1, 3, 7, 64, 255, 256, 270, 480, 1080, 1920, 2160, 3840, 4097, 65535, 100003):
        fx = rng.integers(0, wh + 1, 300000).astype(np.float32)
        r = (rng.integers(0, 1 << 24, fx.size).astype(np.float64) * 2.0 ** -24).astype(np.float32)
        r[:64] = np.float32(0.0)
        r[64:128] = np.float32(2.0 ** -24)
        r[128:192] = np.float32(1.0 - 2.0 ** -24)
        fx[:192] = np.tile(np.array([0, 1, wh - 1 if wh > 1 else 0, wh], np.float32), 48)
        a = (fx + r).astype(np.float32)
        b = np.full_like(a, np.float32(wh))
        out = np.empty_like(a)
        gpu.check(gpu.lib().fr_selftest_ops(0, 9, a.ctypes.data_as(fp), b.ctypes.data_as(fp), a.size,
                                            out.ctypes.data_as(fp)))
        assert _same_bits(out, a / b), wh


def test_fast_sky_parameter_is_bit_identical(gpu):
    """sky_t_fast (the sky blend parameter with guarded core sqrt/division sequences, the
    trace kernel's default; FR_SKY_IEEE builds the plain one) against the plain correctly
    rounded sky_t on the device, bit for bit (op 14 returns the XOR of both results' bits),
    over random directions of every scale, the guards' edges (tiny, zero, -0, denormal
    and huge components) and tiny d.y beside x, z in the fast range."""
    import ctypes as C
    rng = np.random.default_rng(14)
    fp = C.POINTER(C.c_float)
    n = 400000
    scale = (2.0 ** rng.uniform(-70, 70, (3, n))).astype(np.float32)
    v = (rng.standard_normal((3, n)).astype(np.float32) * scale).astype(np.float32)
    edges = np.array([0.0, -0.0, 1e-45, -1e-45, 2.0 ** -100, -(2.0 ** -100), 2.0 ** -101, 2.0 ** -60, 2.0 ** -48,
                      2.0 ** -47, 2.0 ** 62, 2.0 ** 63, 2.0 ** 64, 1.0, -1.0, 3e-39, 1e-30], dtype=np.float32)
    e = np.array(np.meshgrid(edges, edges, edges)).reshape(3, -1)
    # d.y below 2^-100 (normal and denormal) beside x and z that put dot(d, d) in the fast
    # range: the case with no guard of its own
    m = 100000
    tiny = (rng.choice([-1.0, 1.0], m) * 2.0 ** rng.uniform(-149, -100, m)).astype(np.float32)
    big = (rng.standard_normal((2, m)) * 2.0 ** rng.uniform(-47, 62, (2, m))).astype(np.float32)
    t = np.stack([big[0], tiny, big[1]])
    v = np.concatenate([v, e, e[[1, 2, 0]], t], axis=1).astype(np.float32)
    x, y = np.ascontiguousarray(v[0]), np.ascontiguousarray(v[1])  # z of lane i is y[i + 1] (op 14)
    out = np.empty_like(x)
    gpu.check(gpu.lib().fr_selftest_ops(0, 14, x.ctypes.data_as(fp), y.ctypes.data_as(fp), x.size,
                                        out.ctypes.data_as(fp)))
    assert not out.view(np.uint32).any(), int(np.count_nonzero(out.view(np.uint32)))


def _sphere_cases(rng, m):
    """Sphere-test inputs (centre, radius, origin, direction, t_max) of the kinds the kernel
    meets and the fast root's guard edges; rows of 16 f32 (op 16's layout)."""
    f32 = np.float32

    def unit(v):
        return v / np.linalg.norm(v, axis=0)

    fams = []
    # scatter rays: origin on the surface, direction n + a unit-ball point (lambertian)
    c = rng.uniform(-20, 20, (3, m)); r = 10.0 ** rng.uniform(-2, 2, m); n = unit(rng.standard_normal((3, m)))
    o = c + r * n; d = n + unit(rng.standard_normal((3, m))) * rng.uniform(0, 1, m) ** (1 / 3)
    fams.append((c, r, o, d, np.where(rng.uniform(size=m) < 0.5, np.finfo(f32).max, rng.uniform(0.001, 100, m))))
    # camera-like rays from anywhere at any scale
    c = rng.uniform(-50, 50, (3, m)); r = 10.0 ** rng.uniform(-2, 2, m); o = rng.uniform(-10, 10, (3, m))
    d = unit(c - o + rng.standard_normal((3, m)) * r) * 10.0 ** rng.uniform(-3, 1, m)
    fams.append((c, r, o, d, np.full(m, np.finfo(f32).max)))
    # rays leaving spheres they start outside of or near (the behind-the-origin skip)
    c = rng.uniform(-50, 50, (3, m)); r = 10.0 ** rng.uniform(-2, 2, m)
    o = c + unit(rng.standard_normal((3, m))) * r * rng.uniform(0.5, 1.5, m)
    d = unit(o - c + rng.standard_normal((3, m)) * r * rng.uniform(0, 2, m)) * 10.0 ** rng.uniform(-3, 1, m)
    fams.append((c, r, o, d, np.full(m, np.finfo(f32).max)))
    # every component of random sign and exponent (the guards' edges: a, b, disc ranges)
    v = rng.standard_normal((11, m)) * 2.0 ** rng.uniform(-80, 80, (11, m))
    fams.append((v[0:3], np.abs(v[3]), v[4:7], v[7:10], np.where(v[10] > 0, np.finfo(f32).max, np.abs(v[10]))))
    # a and b across the guard bounds 2^-60 / 2^60 and 2^40
    c = rng.uniform(-1, 1, (3, m)) * 2.0 ** rng.uniform(0, 45, m); r = np.abs(c[0]) * rng.uniform(0.1, 2, m)
    o = rng.standard_normal((3, m)); d = unit(c - o + rng.standard_normal((3, m))) * 2.0 ** rng.uniform(-34, 34, m)
    fams.append((c, r, o, d, np.full(m, np.finfo(f32).max)))
    # grazing rays: disc near 0 (tiny and denormal discriminants)
    c = rng.uniform(-20, 20, (3, m)); r = 10.0 ** rng.uniform(-2, 2, m); dh = unit(rng.standard_normal((3, m)))
    pp = unit(np.cross(dh.T, rng.standard_normal((m, 3))).T)
    o = c - 10 * r * dh + r * (1 + rng.uniform(-1e-6, 1e-6, m)) * pp
    fams.append((c, r, o, dh * 10.0 ** rng.uniform(-2, 2, m), np.full(m, np.finfo(f32).max)))
    # the near root at t ~ 0.001 (t_min) and the far root at t ~ t_max
    c = rng.uniform(-20, 20, (3, m)); r = 10.0 ** rng.uniform(-1, 1, m); dh = unit(rng.standard_normal((3, m)))
    s = 10.0 ** rng.uniform(-1, 1, m); o = c - dh * (r + 0.001 * s * rng.uniform(0.999, 1.001, m))
    tfar = (2 * r + 0.001 * s) / s
    fams.append((c, r, o, dh * s, tfar * rng.uniform(1 - 1e-6, 1 + 1e-6, m)))
    rows = []
    for c, r, o, d, tm in fams:
        a = np.zeros((m, 16), dtype=f32)
        a[:, 0:3] = c.T; a[:, 3] = r; a[:, 4:7] = o.T; a[:, 7:10] = d.T; a[:, 10] = tm
        rows.append(a)
    return np.concatenate(rows)


def test_sphere_root_fast_is_bit_identical(gpu):
    """The kernel's sphere test (rt_core.h sphere_root_fast: core sqrt and div_rn with the
    segment's 1/a where the guards hold) against sphere_root's correctly rounded sqrt and
    divisions (shapes/sphere.rs:23-51's arithmetic) on the device: same verdict and the same
    t bits for every case (op 16)."""
    import ctypes as C
    rng = np.random.default_rng(16)
    fp = C.POINTER(C.c_float)
    for _ in range(4):
        cases = _sphere_cases(rng, 100000).astype(np.float32)
        x = np.ascontiguousarray(cases.reshape(-1))
        out = np.empty_like(x)
        gpu.check(gpu.lib().fr_selftest_ops(0, 16, x.ctypes.data_as(fp), x.ctypes.data_as(fp), x.size,
                                            out.ctypes.data_as(fp)))
        bad = out.reshape(-1, 16)[:, 0]
        assert not bad.any(), (int(np.count_nonzero(bad == 1)), int(np.count_nonzero(bad == 2)),
                               cases[np.nonzero(bad)[0][:3]].tolist())


def test_device_schlick_unit_and_u8_match_oracle(gpu):
    import ctypes as C
    rng = np.random.default_rng(2)
    c = rng.uniform(-0.2, 1.2, 4000).astype(np.float32)
    ri = np.full_like(c, np.float32(1.3))
    fp = C.POINTER(C.c_float)
    out = np.empty_like(c)
    gpu.check(gpu.lib().fr_selftest_ops(0, 5, c.ctypes.data_as(fp), ri.ctypes.data_as(fp), c.size,
                                        out.ctypes.data_as(fp)))
    want = np.array([O.vec3(12, (x, 1.3, 0))[0] for x in c[:500]], dtype=np.float32)
    assert _same_bits(out[:500], want)
    x, y = rng.standard_normal(4000).astype(np.float32), rng.standard_normal(4000).astype(np.float32)
    gpu.check(gpu.lib().fr_selftest_ops(0, 7, x.ctypes.data_as(fp), y.ctypes.data_as(fp), x.size,
                                        out.ctypes.data_as(fp)))
    want = np.array([O.vec3(9, (a, b, 1.0))[0] for a, b in zip(x[:500], y[:500])], dtype=np.float32)
    assert _same_bits(out[:500], want)
    v = np.concatenate([np.linspace(-1, 2, 3000), [np.nan, np.inf, -np.inf, 1.0, 0.999999]]).astype(np.float32)
    out = np.empty_like(v)
    gpu.check(gpu.lib().fr_selftest_ops(0, 6, v.ctypes.data_as(fp), v.ctypes.data_as(fp), v.size,
                                        out.ctypes.data_as(fp)))
    with np.errstate(invalid="ignore"):
        s = np.sqrt(v) * np.float32(255.0)
    want = np.where(~(s > 0), 0, np.where(s >= 255, 255, np.trunc(np.nan_to_num(s)))).astype(np.float32)
    assert np.array_equal(out, want)


@pytest.mark.parametrize("seed,pixel,sample", [(0x5EED, 0, 0), (0x5EED, 2073599, 255), (7, 99, 1), (2 ** 63, 5, 9)])
def test_device_rng_matches_oracle(gpu, seed, pixel, sample):
    import ctypes as C
    out = (C.c_uint32 * 200)()
    gpu.check(gpu.lib().fr_selftest_rng(0, seed, pixel, sample, 200, out))
    assert list(out) == list(O.rng_stream(seed, pixel, sample, 200))


# ---- images -----------------------------------------------------------------------

def _product_scene(fr, spec, w, h):
    kind, name = spec.split(":")
    if kind == "builtin":
        return fr.Scene.builtin(int(name), w, h)
    return fr.Scene.from_file(fr.scene_path(name), w, h)


@pytest.mark.parametrize("name", sorted(G.CASES))
def test_golden_cases(gpu, name):
    spec, w, h, spp, depth, seed = G.CASES[name]
    sc = _product_scene(gpu, spec, w, h)
    mean, u8, st = gpu.render(sc, sc.camera, w, h, spp, depth, seed)
    ref = np.load(os.path.join(GOLDEN, f"{name}.npz"))
    cnt = {"segments": int(ref["counters"][0]), "hits": int(ref["counters"][1])}
    assert_parity(mean, u8, st, ref["mean"], ref["u8"], cnt)
    assert st["samples"] == int(ref["counters"][2])


def random_scene(seed, n=12):
    """Every primitive kind and material, placed around the default camera."""
    r = np.random.default_rng(seed)
    prims = []
    for i in range(n):
        kind = r.choice([S.SPHERE, S.SPHERE, S.PLANE, S.AABB, S.OBB, S.STUB, S.TRIANGLE, S.TRIANGLE])
        mat = int(r.integers(0, 5))
        col = r.uniform(0.1, 1.0, 3)
        fuzz = float(r.uniform(0, 1))
        c = r.uniform(-2, 2, 3) + np.array([0, 0, -2.5])
        if kind == S.SPHERE:
            prims.append(S.sphere(c, r.uniform(0.2, 1.2), mat, col, fuzz))
        elif kind == S.PLANE:
            o = np.zeros(3)
            o[r.integers(0, 3)] = r.choice([-1.0, 1.0])
            if r.uniform() < 0.3:
                o = r.standard_normal(3)
            prims.append(S.plane(c, o, r.uniform(0.5, 4, 3), mat, col, fuzz))
        elif kind == S.AABB:
            hsz = r.uniform(0.1, 1.0, 3)
            prims.append(S.prim(S.AABB, mat, col, fuzz, list(c - hsz) + list(c + hsz)))
        elif kind == S.OBB:
            q = r.standard_normal(4)
            q /= np.linalg.norm(q)
            ax = S.quat_axes(*q)
            prims.append(S.prim(S.OBB, mat, col, fuzz, list(c) + list(ax[0]) + list(ax[1]) + list(ax[2])
                                + list(r.uniform(0.1, 1.0, 3))))
        elif kind == S.TRIANGLE:
            v = [list(c + r.uniform(-1.2, 1.2, 3)) for _ in range(3)]
            prims.append(S.prim(S.TRIANGLE, mat, col, fuzz, v[0] + v[1] + v[2]))
        else:
            prims.append(S.prim(S.STUB, mat, col, fuzz))
    prims.append(S.sphere((0.0, -100.5, -1.0), 100.0, 0, (0.5, 0.5, 0.5), 0.0))
    return prims


@pytest.mark.parametrize("seed", range(8))
def test_random_scenes_all_kinds_and_materials(gpu, seed):
    w, h, spp, depth = 40, 24, 3, 8
    prims = random_scene(seed)
    sc = gpu.Scene.from_prims(prims)
    cam = gpu.camera_new(w, h)
    if seed % 2:
        gpu.camera_orbit(cam, (0.4 * seed, 0.1, -2.0))
    ocam = O.camera_new(w, h)
    if seed % 2:
        O.camera_orbit(ocam, (0.4 * seed, 0.1, -2.0))
    mean, u8, st = gpu.render(sc, cam, w, h, spp, depth, seed=1000 + seed)
    omean, ou8, ocnt, _ = O.render(prims, ocam, w, h, spp, depth, seed=1000 + seed, threads=8)
    assert_parity(mean, u8, st, omean, ou8, ocnt)


@pytest.mark.parametrize("seed", [2, 3, 4, 5])
def test_diffuse_only_scenes(gpu, seed):
    """Scenes without metal or dielectric run the diffuse-only shading step (trace_kernel
    MAT = 1) — here the general-kind kernel with planes, stubs, triangles and light (whose
    attenuation is 1, sphere.rs:147-152) — against the oracle."""
    w, h, spp, depth = 40, 24, 4, 8
    prims = random_scene(seed)
    for q in prims:
        if q["material"] in (S.METAL, S.DIELECTRIC):
            q["material"] = S.LIGHT if seed % 2 else S.LAMBERTIAN
    assert len(prims) <= 15
    sc = gpu.Scene.from_prims(prims)
    mean, u8, st = gpu.render(sc, gpu.camera_new(w, h), w, h, spp, depth, seed=300 + seed)
    omean, ou8, ocnt, _ = O.render(prims, O.camera_new(w, h), w, h, spp, depth, seed=300 + seed, threads=8)
    assert_parity(mean, u8, st, omean, ou8, ocnt)


@pytest.mark.parametrize("shards", [2, 3, 8])
def test_row_shards_stitch_bit_exactly(gpu, shards):
    w, h, spp, depth = 100, 50, 4, 8  # H % 8 != 0: last strip is partial
    sc = gpu.Scene.from_file(gpu.scene_path("scene_08"), w, h)
    full, fu8, fst = gpu.render(sc, sc.camera, w, h, spp, depth)
    mean = np.full_like(full, np.nan)
    u8 = np.zeros_like(fu8)
    seg = 0
    for k in range(shards):
        m, u, st = gpu.render(sc, sc.camera, w, h, spp, depth, shard_index=k, shard_count=shards)
        rows = [y for y in range(h) if (y // 8) % shards == k]
        assert np.isnan(m[[y for y in range(h) if y not in rows]]).all()  # other shards untouched
        mean[rows], u8[rows] = m[rows], u[rows]
        seg += st["segments"]
    assert np.array_equal(mean.view(np.uint32), full.view(np.uint32)) and np.array_equal(u8, fu8)
    assert seg == fst["segments"]


def test_multi_device_api_with_one_device(gpu):
    w, h = 48, 40
    sc = gpu.Scene.from_file(gpu.scene_path("scene_08"), w, h)
    a, au, _ = gpu.render(sc, sc.camera, w, h, 2, 8)
    b, bu, _ = gpu.render(sc, sc.camera, w, h, 2, 8, n_gpus=1)
    assert np.array_equal(a, b) and np.array_equal(au, bu)


@pytest.mark.parametrize("n,jit", [(2, False), (8, False), (2, "wait"), (8, "wait")])
def test_multi_context_matches_one_device_bit_for_bit(gpu, n, jit):
    """fr_mctx (tracer.rs:83-134's row tiling, one context per shard) with every entry on
    device 0: the stitched frame equals the N = 1 render bit for bit, frame after frame, and
    the contexts' device buffers and the page-locked host frame stay the same across
    frames (nothing is allocated per frame). jit: every context runs the scene-specialised
    kernel (one module per device, shared by its contexts)."""
    w, h, spp, depth = 100, 70, 20, 8  # H % 8 != 0: the last strip is partial
    sc = gpu.Scene.from_file(gpu.scene_path("scene_08"), w, h)
    ref, ref_u8, ref_st = gpu.render(sc, sc.camera, w, h, spp, depth)
    m = gpu.MultiContext([0] * n)
    p = gpu.make_params(w, h, spp, depth, scene_jit=jit)
    bufs, hostp = None, None
    for _ in range(3):
        m.render(sc, sc.camera, p)
        st = m.sync()
        mean, u8 = m.frame()
        assert np.array_equal(mean.view(np.uint32), ref.view(np.uint32)) and np.array_equal(u8, ref_u8)
        assert (st["segments"], st["hits"], st["scatters"], st["samples"]) == \
            (ref_st["segments"], ref_st["hits"], ref_st["scatters"], ref_st["samples"])
        b = [m.context(i).device_buffers() for i in range(n)]
        hp = m.frame_ptrs()
        assert bufs is None or (b == bufs and hp == hostp)
        bufs, hostp = b, hp
    m.close()


def test_launch_log_times_every_launch(gpu, monkeypatch):
    """fr_ctx_trace_log: HIP-event durations of every trace launch and every render across
    streamed frames (bench.py averages them), here with two passes per frame, and the same
    events as a timeline (tools/frame_gaps.py)."""
    monkeypatch.setenv("FR_PIPELINE", "2")
    w, h = 64, 40
    sc = gpu.Scene.from_file(gpu.scene_path("scene_08"), w, h)
    ctx = gpu.RenderContext(0)
    p = gpu.make_params(w, h, 40, 8)
    ctx.render(sc, sc.camera, p)
    ctx.sync()
    ctx.trace_log(True)
    for _ in range(3):
        ctx.render(sc, sc.camera, p)
    st = ctx.sync()
    launches, frames = ctx.trace_log_read(), ctx.trace_log_read(frames=True)
    assert st["trace_launches"] == 2
    assert len(launches) == 6 and len(frames) == 3
    assert all(t > 0 for t in launches) and all(f >= 0.5 * (a + b) for f, a, b in zip(frames, launches[::2],
                                                                                      launches[1::2]))
    # the same entries as a timeline (which 2 / 3): (start, end) from the first launch's
    # start; each pair's length is the duration above, launches and frames in order
    tl, ftl = ctx.trace_log_read(timeline=True), ctx.trace_log_read(frames=True, timeline=True)
    assert len(tl) == 6 and len(ftl) == 3 and tl[0][0] == 0.0
    for (a, b), dur in zip(tl, launches):
        assert b >= a and abs((b - a) - dur) <= 1e-3 * max(1.0, dur)
    for i in range(3):  # a render's span holds both of its passes
        passes = tl[2 * i:2 * i + 2]
        assert ftl[i][0] <= min(a for a, _ in passes) + 1e-3 and ftl[i][1] >= max(b for _, b in passes) - 1e-3
    ctx.trace_log(False)
    ctx.render(sc, sc.camera, p)
    ctx.sync()
    assert len(ctx.trace_log_read()) == 6  # logging stopped
    ctx.close()


def test_update_pixels_outlive_the_model(gpu):
    """update() returns a view of page-locked memory; the view keeps that memory alive after
    the model is closed and collected (no use-after-free)."""
    import gc
    m = gpu.create_model(40, 30)
    pix = gpu.update(m, 0b001000, 0.1)
    want = pix.copy()
    m.close()
    del m
    gc.collect()
    others = [gpu.PinnedFrame(40, 30) for _ in range(4)]  # would reuse freed pages
    for o in others:
        o.u8[:] = 7
    assert np.array_equal(pix, want)


@pytest.mark.parametrize("case", ["spp1", "depth0", "depth64", "empty", "stubs", "tiny"])
def test_edge_cases(gpu, case):
    w, h, spp, depth, prims = 24, 16, 2, 8, S.BUILTIN[2]()
    if case == "spp1":
        spp = 1
    elif case == "depth0":
        depth = 0
    elif case == "depth64":
        depth, prims = 64, S.BUILTIN[3]()
    elif case == "empty":
        prims = []
    elif case == "stubs":
        prims = [S.prim(S.STUB)] * 3
    elif case == "tiny":
        w, h = 1, 1
    sc = gpu.Scene.from_prims(prims)
    cam, ocam = gpu.camera_new(w, h), O.camera_new(w, h)
    mean, u8, st = gpu.render(sc, cam, w, h, spp, depth)
    omean, ou8, ocnt, _ = O.render(prims, ocam, w, h, spp, depth)
    assert_parity(mean, u8, st, omean, ou8, ocnt)


@pytest.mark.parametrize("spp", [16, 17, 20, 21, 32, 33, 47, 48])
def test_last_block_sub_block_streams(gpu, spp):
    """Around the stream layout's edges: spp = 16 (one block, no sub-blocks), a last block
    of 1, 4, 5, 15 or 16 samples (sub-blocks of 4, the last partial); the sub-block items
    are the queue's last items and land in their block's sample slots."""
    w, h, depth = 40, 24, 8
    sc = gpu.Scene.from_file(gpu.scene_path("scene_08"), w, h)
    mean, u8, st = gpu.render(sc, sc.camera, w, h, spp, depth, seed=spp)
    prims, (frm, at, vup, fov) = S.load_json(open(gpu.scene_path("scene_08")).read())
    cam = O.camera_look(frm, at, vup, fov, 0.1, w, h)
    omean, ou8, ocnt, _ = O.render(prims, cam, w, h, spp, depth, seed=spp, threads=8)
    assert_parity(mean, u8, st, omean, ou8, ocnt)


@pytest.mark.parametrize("wgs,scene,w,h,spp,depth", [(1, "scene_08", 64, 40, 40, 8), (3, "scene_01", 48, 32, 20, 8),
                                                    (1, "scene_02", 40, 24, 3, 12), (2, "scene_08", 72, 16, 1, 4)])
def test_small_grid_claims_many_batches(gpu, wgs, scene, w, h, spp, depth, monkeypatch):
    """FR_MAX_WGS caps the persistent grid, so each wave claims many 64-item batches, one
    or a few lanes at a time, across sample blocks and across partly used batches: the
    claim step's lane permutes (stream, pixel, block from the seeding lane) and the queue
    tail run at a size the oracle renders whole."""
    monkeypatch.setenv("FR_MAX_WGS", str(wgs))
    sc = gpu.Scene.from_file(gpu.scene_path(scene), w, h)
    mean, u8, st = gpu.render(sc, sc.camera, w, h, spp, depth)
    prims, (frm, at, vup, fov) = S.load_json(open(gpu.scene_path(scene)).read())
    cam = O.camera_look(frm, at, vup, fov, 0.1, w, h)
    omean, ou8, ocnt, _ = O.render(prims, cam, w, h, spp, depth, threads=8)
    assert_parity(mean, u8, st, omean, ou8, ocnt)
    assert st["occupancy"] >= 1


def test_context_reuse_and_scene_edits(gpu):
    w, h = 32, 32
    sc = gpu.Scene.builtin(0, w, h)
    ctx = gpu.RenderContext(0)
    ctx.render(sc, sc.camera, gpu.make_params(w, h, 2, 8))
    ctx.sync()
    a, _ = ctx.download(w, h)
    sc.translate(0, (-1.0, 0.0, 0.0))
    sc.rotate(0, (-1.0, 0.0, 0.0))  # the scene's device copy must be refreshed
    ctx.render(sc, sc.camera, gpu.make_params(w, h, 2, 8))
    st = ctx.sync()
    b, bu = ctx.download(w, h)
    omean, ou8, ocnt, _ = O.render(S.BUILTIN[3](), O.camera_new(w, h), w, h, 2, 8)
    assert_parity(b, bu, st, omean, ou8, ocnt)
    assert not np.array_equal(a, b)
    ctx.close()


@pytest.mark.parametrize("shard,pipe", [((0, 1), "0"), ((1, 3), "0"), ((0, 1), "1"), ((1, 3), "1"), ((0, 1), "2"),
                                        ((1, 3), "2"), ((0, 1), ""), ((1, 3), "")])
def test_streamed_frames_match_the_oracle(gpu, shard, pipe, monkeypatch):
    """bench.py's loop: frames enqueued back to back on one context, each followed by its
    asynchronous gather into the same pinned host frame, one sync after the last. The
    streams alone order the frames, so the host frame holds the last frame's strips
    exactly, and the counters are that frame's. pipe "1": the frame pipeline (FR_FRAME_PIPE,
    frame k+1's trace beside frame k's sum); "2": consecutive traces may overlap too; "":
    the default choice."""
    monkeypatch.setenv("FR_FRAME_PIPE", pipe)
    w, h, spp, depth = 64, 40, 20, 8
    sc = gpu.Scene.from_file(gpu.scene_path("scene_08"), w, h)
    prims, (frm, at, vup, fov) = S.load_json(open(gpu.scene_path("scene_08")).read())
    cam = O.camera_look(frm, at, vup, fov, 0.1, w, h)
    omean, ou8, ocnt, _ = O.render(prims, cam, w, h, spp, depth, threads=8, shard_index=shard[0],
                                   shard_count=shard[1])
    rows = [y for y in range(h) if (y // 8) % shard[1] == shard[0]]
    p = gpu.make_params(w, h, spp, depth, shard_index=shard[0], shard_count=shard[1])
    ctx = gpu.RenderContext(0)
    frame = gpu.PinnedFrame(w, h)
    for _ in range(4):
        ctx.render(sc, sc.camera, p)
        ctx.download_async(frame)
    st = ctx.sync()
    ctx.wait()
    assert_parity(frame.mean.copy(), frame.u8.copy(), st, omean, ou8, ocnt, rows=rows)
    frame.close()
    ctx.close()


@pytest.mark.parametrize("jit,pipe,slots", [(False, "1", None), ("wait", "1", None), (False, "2", None),
                                           ("wait", "2", None), (False, "1", "3"), ("wait", "2", "4")])
def test_pipelined_frames_of_different_seeds(gpu, jit, pipe, slots, monkeypatch):
    """Five frames of different seeds enqueued back to back with the frame pipeline, each
    gathered into its own pinned frame: every gather holds its own frame (the frame slots,
    two by default, FR_FRAME_SLOTS 3 or 4, are reused in turn), equal to the frame rendered
    alone."""
    w, h, spp, depth = 64, 40, 33, 8
    sc = gpu.Scene.from_file(gpu.scene_path("scene_08"), w, h)
    seeds = [3, 4, 5, 6, 7]
    refs = [gpu.render(sc, sc.camera, w, h, spp, depth, seed=sd) for sd in seeds]
    monkeypatch.setenv("FR_FRAME_PIPE", pipe)
    if slots:
        monkeypatch.setenv("FR_FRAME_SLOTS", slots)
    ctx = gpu.RenderContext(0)
    frames = [gpu.PinnedFrame(w, h) for _ in seeds]
    for sd, fr_ in zip(seeds, frames):
        ctx.render(sc, sc.camera, gpu.make_params(w, h, spp, depth, seed=sd, scene_jit=jit))
        ctx.download_async(fr_)
    st = ctx.sync()
    ctx.wait()
    for (m, u, _), fr_ in zip(refs, frames):
        assert np.array_equal(fr_.mean.view(np.uint32), m.view(np.uint32)) and np.array_equal(fr_.u8, u)
    assert (st["segments"], st["hits"], st["scatters"]) == (refs[-1][2]["segments"], refs[-1][2]["hits"],
                                                            refs[-1][2]["scatters"])
    for fr_ in frames:
        fr_.close()
    ctx.close()


def test_update_and_save_image_mirror(gpu, tmp_path):
    w, h = 40, 30
    m = gpu.create_model(w, h)
    pix = gpu.update(m, 0b001000, 0.25)  # A key: orbit by +0.25 rad
    assert pix.shape == (w * h * 3,) and pix.dtype == np.uint8
    ocam = O.camera_orbit(O.camera_new(w, h), (0.25, 0.0, 0.0))
    assert np.array_equal(m.scene.camera.to_array(), O.camera_to_array(ocam))
    seed = m.seed ^ (0x9E3779B97F4A7C15 * 1 & 0xFFFFFFFFFFFFFFFF)
    _, ou8, _, _ = O.render(S.BUILTIN[0](), ocam, w, h, 1, 50, seed=seed)
    assert np.array_equal(pix.reshape(h, w, 3), ou8)
    out = tmp_path / "basic.png"
    mean, u8, st = gpu.save_image(m, 3, str(out))
    assert out.read_bytes()[:8] == b"\x89PNG\r\n\x1a\n" and st["samples"] == w * h * 3


def test_update_frames_reuse_one_context(gpu):
    """tracer.rs:30-55 as a frame loop: every update() runs on the model's one fr_ctx (same
    handle and the same device output buffers across frames, so no per-frame context or
    buffer allocation), and each 1-spp frame equals the oracle's render of the orbited
    camera with that frame's RNG key."""
    import ctypes as C
    w, h = 40, 30
    m = gpu.create_model(w, h)
    ocam = O.camera_new(w, h)
    handles, buffers = set(), set()
    for frame, keys in enumerate([0b001000, 0b000100, 0b100000, 0b000001, 0b010010]):
        pix = gpu.update(m, keys, 0.1)
        handles.add(m.ctx._h.value)
        buffers.add(m.ctx.device_buffers())
        d = (C.c_float * 3)()
        gpu.check(gpu.lib().fr_update_delta(keys, 0.1, d))
        O.camera_orbit(ocam, list(d))
        assert np.array_equal(m.scene.camera.to_array(), O.camera_to_array(ocam))
        seed = m.seed ^ (0x9E3779B97F4A7C15 * (frame + 1) & 0xFFFFFFFFFFFFFFFF)
        _, ou8, ocnt, _ = O.render(S.BUILTIN[0](), ocam, w, h, 1, 50, seed=seed)
        assert np.array_equal(pix.reshape(h, w, 3), ou8), frame
        assert (m.last_stats["segments"], m.last_stats["hits"]) == (ocnt["segments"], ocnt["hits"])
    assert len(handles) == 1 and len(buffers) == 1
    m.close()


# ---- full-size configurations (BASELINE.json configs) ----------------------------

def _rows(h, step):
    return list(range(0, h, step))


def oracle_threads():
    """CPUs this process can use at once: the affinity mask capped at the cgroup quota
    (the GPU box runs the tests in a 16-CPU quota; more threads than that only contend)."""
    import math
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, math.ceil(int(q) / int(per))))
    except Exception:
        pass
    return max(1, n)


def _progress(tag):
    import time
    t0 = time.time()

    def f(done, total):
        print(f"[{tag}] oracle rows {done}/{total} ({time.time() - t0:.0f}s)", flush=True)
    return f


def test_c1_full_frame(gpu):
    """BASELINE config C1 (scene_01 at 256x256, 4 spp, 4 bounces), the reference's
    CPU-runnable case, rendered whole on the GPU and by the oracle: all 65,536 pixels
    (262,144 samples) compared, with the segment, hit and scatter counters."""
    name, w, h, spp, depth = "scene_01", 256, 256, 4, 4
    sc = gpu.Scene.from_file(gpu.scene_path(name), w, h)
    mean, u8, st = gpu.render(sc, sc.camera, w, h, spp, depth)
    assert st["samples"] == w * h * spp == 262144
    prims, (frm, at, vup, fov) = S.load_json(open(gpu.scene_path(name)).read())
    cam = O.camera_look(frm, at, vup, fov, 0.1, w, h)
    omean, ou8, ocnt, n = O.render(prims, cam, w, h, spp, depth, threads=16)
    assert n == h
    assert_parity(mean, u8, st, omean, ou8, ocnt)
    assert np.array_equal(mean.view(np.uint32), omean.view(np.uint32))


@pytest.mark.slow
def test_c3_headline_frame_in_full(gpu):
    """C3, the config the headline number is quoted on (scene_08 at 1920x1080, 256 spp, 8
    bounces; tracer.rs:160-187's whole image), through the HIP path and the oracle: all
    2,073,600 pixels (530.8 M samples) compared — means within 1e-5 and bit for bit, u8
    identical — and the whole-frame segment, hit and scatter counters equal. Both trace
    kernels: the compiled-in one and the scene-specialised one bench.py runs (DESIGN.md
    §4.8)."""
    name, w, h, spp, depth = "scene_08", 1920, 1080, 256, 8
    sc = gpu.Scene.from_file(gpu.scene_path(name), w, h)
    runs = [gpu.render(sc, sc.camera, w, h, spp, depth, scene_jit=jit) for jit in (False, "wait")]
    assert runs[0][2]["samples"] == w * h * spp == 530841600
    prims, (frm, at, vup, fov) = S.load_json(open(gpu.scene_path(name)).read())
    cam = O.camera_look(frm, at, vup, fov, 0.1, w, h)
    omean, ou8, ocnt = O.render_rows(prims, cam, w, h, spp, depth, range(h), threads=oracle_threads(), chunk=120,
                                     progress=_progress("C3"))
    for mean, u8, st in runs:
        assert ocnt["samples"] == st["samples"]
        assert_parity(mean, u8, st, omean, ou8, ocnt)
        assert np.array_equal(mean.view(np.uint32), omean.view(np.uint32))


@pytest.mark.slow
def test_c2_full_frame(gpu):
    """C2 (scene_01: 43 primitives with a plane, 1920x1080, 64 spp, 8 bounces), the whole
    frame against the oracle: all 2,073,600 pixels (132.7 M samples) within 1e-5 and bit for
    bit, u8 identical, the whole-frame segment, hit and scatter counters equal. Both trace
    kernels: the compiled-in one and the scene-specialised one."""
    name, w, h, spp, depth = "scene_01", 1920, 1080, 64, 8
    sc = gpu.Scene.from_file(gpu.scene_path(name), w, h)
    mean, u8, st = gpu.render(sc, sc.camera, w, h, spp, depth)
    assert st["samples"] == w * h * spp == 132710400
    jm, ju, jst = gpu.render(sc, sc.camera, w, h, spp, depth, scene_jit="wait")
    assert np.array_equal(jm.view(np.uint32), mean.view(np.uint32)) and np.array_equal(ju, u8)
    assert (jst["segments"], jst["hits"], jst["scatters"]) == (st["segments"], st["hits"], st["scatters"])
    prims, (frm, at, vup, fov) = S.load_json(open(gpu.scene_path(name)).read())
    cam = O.camera_look(frm, at, vup, fov, 0.1, w, h)
    omean, ou8, ocnt = O.render_rows(prims, cam, w, h, spp, depth, range(h), threads=oracle_threads(), chunk=60,
                                     progress=_progress("C2"))
    assert ocnt["samples"] == st["samples"]
    assert_parity(mean, u8, st, omean, ou8, ocnt)
    assert np.array_equal(mean.view(np.uint32), omean.view(np.uint32))


@pytest.mark.slow
def test_c4_full_frame_every_shard_through_mctx(gpu, monkeypatch):
    """C4 (scene_08 3840x2160, 1024 spp, 8 bounces, row-tiled across 8 devices) as the
    drop-in renders it: one fr_mctx over 8 contexts (here all on device 0), the scene kernel,
    the whole 8.49 G-sample frame stitched in the page-locked host frame. Against the oracle:
    4 full 3,840-px rows of every shard (spread over its strips), and every one of the 2,160
    rows at every 8th pixel (1.06 G samples: each strip of each shard, so every shard's
    claims, sub-blocks and tiles); the stitched frame's counters equal the sum of the eight
    shard renders'."""
    monkeypatch.setenv("FR_SAMPLE_BUFFER_GB", "12")  # one pass per shard, no frame slots: 8 x 8.5 GB
    w, h, spp, depth, n = 3840, 2160, 1024, 8, 8
    sc = gpu.Scene.from_file(gpu.scene_path("scene_08"), w, h)
    m = gpu.MultiContext([0] * n)
    try:
        m.render(sc, sc.camera, gpu.make_params(w, h, spp, depth, scene_jit="wait"))
        tot = m.sync()
        shard_st = [m.context(i).sync() for i in range(n)]
        assert all(m.context(i).jit_state() == gpu.FR_JIT_USED for i in range(n))
        mean, u8 = m.frame()
    finally:
        m.close()
    assert tot["samples"] == w * h * spp == 8493465600
    for k in ("segments", "hits", "scatters", "samples"):
        assert tot[k] == sum(s[k] for s in shard_st), k
    assert not np.isnan(mean).any() and (mean >= 0).all() and (mean <= 1).all()
    rows = []
    for k in range(n):
        mine = [y for y in range(h) if (y // 8) % n == k]
        rows += [mine[0], mine[len(mine) // 3], mine[(2 * len(mine)) // 3], mine[-1]]
    prims, (frm, at, vup, fov) = S.load_json(open(gpu.scene_path("scene_08")).read())
    cam = O.camera_look(frm, at, vup, fov, 0.1, w, h)
    omean, ou8, _ = O.render_rows(prims, cam, w, h, spp, depth, rows, threads=oracle_threads(), chunk=4,
                                  progress=_progress("C4 all shards"))
    assert_parity(mean, u8, None, omean, ou8, None, rows=rows)
    assert np.array_equal(mean[rows].view(np.uint32), omean[rows].view(np.uint32))
    # every row, every 8th column
    cmean, cu8, ccnt = O.render_rows(prims, cam, w, h, spp, depth, range(h), threads=oracle_threads(), col_step=8,
                                     chunk=240, progress=_progress("C4 every row, col_step 8"))
    assert ccnt["samples"] == h * (w // 8) * spp
    assert_parity(mean[:, ::8], u8[:, ::8], None, cmean[:, ::8], cu8[:, ::8], None)
    assert np.array_equal(mean[:, ::8].view(np.uint32), cmean[:, ::8].view(np.uint32))


# ---- BVH (scenes of >= 48 primitives, <= 32 planes) -------------

def bvh_cost(prims):
    """bvh.cpp's weighted test cost (the BVH is used at >= 48, with >= 48 primitives)."""
    w = {S.TRIANGLE: 2.5, S.OBB: 2.0, S.STUB: 0.0}
    return sum(w.get(p["kind"], 1.0) for p in prims)


def bvh_scene(seed, n=400, dup=True, planes=0):
    """Plane-free random scene of every bounded kind plus stubs; with dup, exact copies
    of earlier primitives later in the list (and of later ones earlier), so exact-t ties
    between list positions occur on every frame."""
    r = np.random.default_rng(seed)
    prims = []
    for i in range(n):
        kind = r.choice([S.SPHERE, S.SPHERE, S.AABB, S.OBB, S.TRIANGLE, S.TRIANGLE, S.STUB])
        mat = int(r.integers(0, 5))
        col = r.uniform(0.1, 1.0, 3)
        fuzz = float(r.uniform(0, 1))
        c = r.uniform(-6, 6, 3) + np.array([0, 0, -8.0])
        if kind == S.SPHERE:
            prims.append(S.sphere(c, r.uniform(0.1, 0.9), mat, col, fuzz))
        elif kind == S.AABB:
            hsz = r.uniform(0.05, 0.8, 3)
            prims.append(S.prim(S.AABB, mat, col, fuzz, list(c - hsz) + list(c + hsz)))
        elif kind == S.OBB:
            q = r.standard_normal(4)
            q /= np.linalg.norm(q)
            ax = S.quat_axes(*q)
            prims.append(S.prim(S.OBB, mat, col, fuzz, list(c) + list(ax[0]) + list(ax[1]) + list(ax[2])
                                + list(r.uniform(0.05, 0.8, 3))))
        elif kind == S.TRIANGLE:
            v = [list(c + r.uniform(-1.0, 1.0, 3)) for _ in range(3)]
            prims.append(S.prim(S.TRIANGLE, mat, col, fuzz, v[0] + v[1] + v[2]))
        else:
            prims.append(S.prim(S.STUB, mat, col, fuzz))
    if dup:
        for j in r.integers(0, n, 20):
            q = dict(prims[int(j)])
            q["material"] = int(r.integers(0, 4))  # same geometry, other material: the winner is visible
            q["color"] = np.asarray(r.uniform(0.1, 1.0, 3), dtype=np.float32)
            if r.uniform() < 0.5:
                prims.append(q)
            else:
                prims.insert(int(r.integers(0, int(j) + 1)), q)
    for _ in range(planes):  # planes cut the list into BVH runs (bvh.h)
        o = np.zeros(3)
        o[r.integers(0, 3)] = r.choice([-1.0, 1.0])
        if r.uniform() < 0.3:
            o = r.standard_normal(3)
        c = r.uniform(-6, 6, 3) + np.array([0, 0, -8.0])
        prims.insert(int(r.integers(0, len(prims) + 1)),
                     S.plane(c, o, r.uniform(0.5, 4, 3), int(r.integers(0, 5)), r.uniform(0.1, 1.0, 3), 0.3))
    prims.append(S.sphere((0.0, -1000.5, -1.0), 1000.0, 0, (0.5, 0.5, 0.5), 0.0))
    return prims


@pytest.mark.parametrize("seed,planes,depth", [(0, 0, 8), (1, 0, 8), (2, 0, 8), (3, 0, 8), (4, 1, 8), (5, 3, 8),
                                               (6, 12, 8), (0, 0, 12), (5, 3, 12), (1, 0, 50), (6, 12, 50)])
def test_bvh_matches_list_order_loop(gpu, seed, planes, depth, monkeypatch):
    """Depth 8 runs the u16-stack BVH kernels (MAXD = 8); 12 and 50 the u32-stack ones
    (MAXD = 0, which place the traversal stack after max_depth levels)."""
    w, h, spp = 48, 32, 3
    prims = bvh_scene(seed, planes=planes)
    assert bvh_cost(prims) >= 48 and len(prims) >= 48  # so the product takes the BVH path
    sc = gpu.Scene.from_prims(prims)
    cam = gpu.camera_new(w, h)
    gpu.camera_orbit(cam, (0.3 * seed, 0.05 * seed, 1.5))
    ocam = O.camera_new(w, h)
    O.camera_orbit(ocam, (0.3 * seed, 0.05 * seed, 1.5))
    mean, u8, st = gpu.render(sc, cam, w, h, spp, depth, seed=77 + seed)
    omean, ou8, ocnt, _ = O.render(prims, ocam, w, h, spp, depth, seed=77 + seed, threads=8)
    assert_parity(mean, u8, st, omean, ou8, ocnt)
    monkeypatch.setenv("FR_BVH", "0")  # the in-order loop gives the same bits
    mean0, u80, st0 = gpu.render(gpu.Scene.from_prims(prims), cam, w, h, spp, depth, seed=77 + seed)
    assert np.array_equal(mean0.view(np.uint32), mean.view(np.uint32)) and st0["hits"] == st["hits"]


@pytest.mark.parametrize("seed,planes,k,depth", [(0, 0, 1, 8), (1, 0, 7, 8), (2, 3, 15, 8), (3, 0, 16, 8),
                                                 (6, 12, 5, 8), (4, 1, 3, 5)])
def test_bvh_attenuation_class_records(gpu, seed, planes, k, depth, monkeypatch):
    """Diffuse BVH scenes with at most 15 distinct attenuations (lambertian colours, light's
    1) run the BVH kernel with 8-B records: a path's winners stored as attenuation classes
    and multiplied out by sum_nib_kernel from the class table; 16 classes
    keep the unwind in the trace kernel. Every kind, stubs, planes between BVH runs and
    list-order ties: against the oracle, the unwinding BVH kernel (FR_DEFER=0) and the
    in-order loop (FR_BVH=0), bit for bit."""
    w, h, spp = 48, 32, 3
    prims = bvh_scene(seed, planes=planes)
    r = np.random.default_rng(100 + seed)
    pal = r.uniform(0.1, 1.0, (k, 3)).astype(np.float32)
    for q in prims:
        q["material"] = S.LIGHT if (k < 15 and r.uniform() < 0.1) else S.LAMBERTIAN
        q["color"] = pal[int(r.integers(0, k))]
        q["fuzz"] = np.float32(0.0)
    sc = gpu.Scene.from_prims(prims)
    cam, ocam = gpu.camera_new(w, h), O.camera_new(w, h)
    gpu.camera_orbit(cam, (0.3 * seed, 0.05 * seed, 1.5))
    O.camera_orbit(ocam, (0.3 * seed, 0.05 * seed, 1.5))
    monkeypatch.delenv("FR_DEFER", raising=False)
    mean, u8, st = gpu.render(sc, cam, w, h, spp, depth, seed=91 + seed)
    omean, ou8, ocnt, _ = O.render(prims, ocam, w, h, spp, depth, seed=91 + seed, threads=8)
    assert_parity(mean, u8, st, omean, ou8, ocnt)
    for env in (("FR_DEFER", "0"), ("FR_BVH", "0")):
        monkeypatch.setenv(*env)
        m0, u0, st0 = gpu.render(gpu.Scene.from_prims(prims), cam, w, h, spp, depth, seed=91 + seed)
        assert np.array_equal(m0.view(np.uint32), mean.view(np.uint32)) and np.array_equal(u0, u8), env
        assert (st0["segments"], st0["hits"]) == (st["segments"], st["hits"]), env
        monkeypatch.delenv(env[0])


def test_bvh_attenuation_class_records_across_passes(gpu, monkeypatch):
    """The class records through the multi-pass path (a sample buffer of one block per pass:
    traces alternate between two streams, sum_nib_kernel carries the running sum): the same
    bits as one pass, for a diffuse three-class BVH scene."""
    w, h, spp, depth = 256, 128, 40, 8
    prims = bvh_scene(9)
    r = np.random.default_rng(109)
    pal = r.uniform(0.1, 1.0, (3, 3)).astype(np.float32)
    for q in prims:
        q["material"] = S.LAMBERTIAN
        q["color"] = pal[int(r.integers(0, 3))]
    cam = gpu.camera_new(w, h)
    one = gpu.render(gpu.Scene.from_prims(prims), cam, w, h, spp, depth, seed=5)
    monkeypatch.setenv("FR_SAMPLE_BUFFER_GB", "0.001")  # 1 MiB: one 4-MiB block per pass
    many = gpu.render(gpu.Scene.from_prims(prims), cam, w, h, spp, depth, seed=5)
    assert many[2]["trace_launches"] == 3, many[2]
    assert np.array_equal(many[0].view(np.uint32), one[0].view(np.uint32)) and np.array_equal(many[1], one[1])
    assert (many[2]["segments"], many[2]["hits"]) == (one[2]["segments"], one[2]["hits"])


@pytest.mark.parametrize("layout", ["same", "line", "pairs"])
def test_bvh_degenerate_trees_keep_list_order_ties(gpu, layout, monkeypatch):
    """Trees the SAH sweep cannot separate: 64 identical spheres (every hit a tie: the list's
    first wins), 64 spheres on one line, and 32 pairs of coincident spheres of different
    colours. The BVH walk against the oracle and the in-order loop, bit for bit."""
    w, h, spp, depth = 40, 24, 3, 8
    r = np.random.default_rng(11)
    prims = []
    for i in range(64):
        c = {"same": (0.0, 0.0, -3.0), "line": (0.3 * i - 9.6, 0.0, -6.0),
             "pairs": tuple(r.uniform(-3, 3, 2)) + (-7.0,) if i % 2 == 0 else None}[layout]
        if c is None:
            c = prims[-1]["g"][:3]  # the pair's second sphere: the same centre
        prims.append(S.sphere(tuple(float(v) for v in c), 0.6, i % 4, tuple(float(v) for v in r.uniform(0.2, 1, 3)), 0.1))
    prims.append(S.sphere((0.0, -100.5, -1.0), 100.0, 0, (0.5, 0.5, 0.5), 0.0))
    assert bvh_cost(prims) >= 48 and len(prims) >= 48
    sc = gpu.Scene.from_prims(prims)
    cam, ocam = gpu.camera_new(w, h), O.camera_new(w, h)
    mean, u8, st = gpu.render(sc, cam, w, h, spp, depth, seed=5)
    omean, ou8, ocnt, _ = O.render(prims, ocam, w, h, spp, depth, seed=5, threads=8)
    assert_parity(mean, u8, st, omean, ou8, ocnt)
    monkeypatch.setenv("FR_BVH", "0")
    mean0, _, st0 = gpu.render(gpu.Scene.from_prims(prims), cam, w, h, spp, depth, seed=5)
    assert np.array_equal(mean0.view(np.uint32), mean.view(np.uint32)) and st0["hits"] == st["hits"]


@pytest.mark.parametrize("classes", [None, 4])
def test_bvh_far_origins_from_stale_plane_records(gpu, classes, monkeypatch):
    """Planes listed after the other primitives, small and in every orientation: a plane
    whose denominator gate passes (plane.rs:26) but whose bounds test fails still writes
    t (plane.rs:27-40), so the scatter origin p = o + t_stale d of the earlier winner can
    lie thousands of scene extents away, where the BVH's node cull is not conservative.
    Waves with such an origin walk the list in order (render.hip); the image must equal
    the list-order loop (FR_BVH=0) and the oracle bit for bit. classes=4: the scene made
    diffuse with four colours, so the BVH kernel with attenuation-class records runs it."""
    prims = bvh_scene(7, n=300)[:-1]  # no ground sphere: the scene extent stays small
    r = np.random.default_rng(7)
    for _ in range(16):
        o = r.standard_normal(3)
        c = r.uniform(-6, 6, 3) + np.array([0, 0, -8.0])
        prims.append(S.plane(c, o, r.uniform(0.2, 1.0, 3), int(r.integers(0, 2)), r.uniform(0.1, 1.0, 3), 0.3))
    if classes:
        pal = r.uniform(0.1, 1.0, (classes, 3)).astype(np.float32)
        for q in prims:
            q["material"] = S.LAMBERTIAN
            q["color"] = pal[int(r.integers(0, classes))]
    assert bvh_cost(prims) >= 48
    w, h, spp, depth = 48, 32, 6, 8
    cam = gpu.camera_new(w, h)
    gpu.camera_orbit(cam, (0.4, 0.1, 1.5))
    ocam = O.camera_new(w, h)
    O.camera_orbit(ocam, (0.4, 0.1, 1.5))
    mean, u8, st = gpu.render(gpu.Scene.from_prims(prims), cam, w, h, spp, depth, seed=31)
    omean, ou8, ocnt, _ = O.render(prims, ocam, w, h, spp, depth, seed=31, threads=8)
    assert_parity(mean, u8, st, omean, ou8, ocnt)
    monkeypatch.setenv("FR_BVH", "0")
    mean0, _, st0 = gpu.render(gpu.Scene.from_prims(prims), cam, w, h, spp, depth, seed=31)
    assert np.array_equal(mean0.view(np.uint32), mean.view(np.uint32)) and st0["hits"] == st["hits"]


@pytest.mark.parametrize("depth", [8, 12, 50])
def test_bvh_generator_10k_spheres_small(gpu, depth, monkeypatch):
    """C5's scene (tools/gen_scene.py --count 10000 --mesh sphere) at a size the oracle's
    brute-force loop finishes quickly; depth 12 and 50 run the u32-stack kernels."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_scene", os.path.join(ROOT, "tools", "gen_scene.py"))
    gs = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gs)
    text = gs.dumps(gs.generator_scene(10000, "sphere"))
    w, h, spp = 48, 27, 2
    sc = gpu.Scene.from_json(text, w, h)
    assert len(sc) == 10000
    mean, u8, st = gpu.render(sc, sc.camera, w, h, spp, depth)
    prims, (frm, at, vup, fov) = S.load_json(text)
    cam = O.camera_look(frm, at, vup, fov, 0.1, w, h)
    omean, ou8, ocnt, _ = O.render(prims, cam, w, h, spp, depth, threads=16)
    assert_parity(mean, u8, st, omean, ou8, ocnt)
    assert st["hits"] > 0
    # the generator's spheres are all lambertian: the diffuse-only BVH kernels ran; the
    # general shading step (FR_MAT=0) gives the same bits
    monkeypatch.setenv("FR_MAT", "0")
    mean0, u80, st0 = gpu.render(sc, sc.camera, w, h, spp, depth)
    assert np.array_equal(mean0.view(np.uint32), mean.view(np.uint32)) and st0["segments"] == st["segments"]


@pytest.mark.parametrize("scene,spp", [("scene_08", 3), ("scene_08", 37), ("random", 5)])
def test_record_formats_are_bit_identical(gpu, scene, spp, monkeypatch):
    """The deferred unwind stores 8-B records (4-bit winners) for scenes of <= 15
    primitives and 12-B records (u8 winners) above; FR_DEFER=1 forces the 12-B form and
    FR_DEFER=0 the unwind in the trace kernel; FR_MAT=0 the general shading step where a
    scene has no metal or dielectric (scene_08). All give the same bits."""
    w, h = 48, 32
    if scene == "random":
        prims = [p for p in random_scene(5) if p["kind"] != S.PLANE]
        sc = gpu.Scene.from_prims(prims)
        cam = gpu.camera_new(w, h)
    else:
        sc = gpu.Scene.from_file(gpu.scene_path(scene), w, h)
        cam = sc.camera
    assert len(sc) <= 15
    monkeypatch.delenv("FR_DEFER", raising=False)
    monkeypatch.delenv("FR_MAT", raising=False)
    ref = gpu.render(sc, cam, w, h, spp, 8)
    for env in (("FR_DEFER", "1"), ("FR_DEFER", "0"), ("FR_MAT", "0")):
        monkeypatch.delenv("FR_DEFER", raising=False)
        monkeypatch.setenv(*env)
        mean, u8, st = gpu.render(sc, cam, w, h, spp, 8)
        assert np.array_equal(mean.view(np.uint32), ref[0].view(np.uint32)) and np.array_equal(u8, ref[1]), env
        assert (st["segments"], st["hits"], st["scatters"]) == (ref[2]["segments"], ref[2]["hits"], ref[2]["scatters"])


@pytest.mark.parametrize("spp", [3, 21])
def test_bvh_sample_staging_is_bit_identical(gpu, spp, monkeypatch):
    """BVH kernels store each sample directly by default; FR_BVH_STAGE=2 stages 2 samples per
    store when the LDS allows it (KF_STAGE, the C5 scene), 1 even at a lower residency. Same
    bits, whole sub-blocks and partial groups (spp 3, 21) included."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_scene", os.path.join(ROOT, "tools", "gen_scene.py"))
    gs = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gs)
    text = gs.dumps(gs.generator_scene(10000, "sphere"))
    w, h = 64, 40
    sc = gpu.Scene.from_json(text, w, h)
    monkeypatch.delenv("FR_BVH_STAGE", raising=False)
    ref = gpu.render(sc, sc.camera, w, h, spp, 8)
    for mode in ("1", "2"):
        monkeypatch.setenv("FR_BVH_STAGE", mode)
        mean, u8, st = gpu.render(sc, sc.camera, w, h, spp, 8)
        assert np.array_equal(mean.view(np.uint32), ref[0].view(np.uint32)) and np.array_equal(u8, ref[1])
        assert (st["segments"], st["hits"]) == (ref[2]["segments"], ref[2]["hits"])


def test_bvh_far_scene_axis_parallel_bounces(gpu, monkeypatch):
    """A scene ~40000 units from the origin: a lambertian bounce ((p + n) + r) - p there has
    an exact-zero direction component every few hundred scatters (ulp(p) = 2^-8), so 1/d
    is +-inf. The node cull must keep boxes such a ray is inside (render.hip clamps the
    cull's reciprocal, bvh.h kBvhInvClamp); C5's spheres at y ~ 5000 hit the same case."""
    r = np.random.default_rng(11)
    base = np.array([40000.0, 40000.0, 40000.0])
    prims = []
    for i in range(7):
        for j in range(7):
            for k in range(6):
                c = base + np.array([4.0 * i - 12, 4.0 * j - 12, 4.0 * k + 10]) + r.uniform(-0.5, 0.5, 3)
                mat = int(r.choice([0, 0, 0, 1, 2]))
                if (i + j + k) % 3 == 0:
                    h = r.uniform(0.6, 1.6, 3)
                    prims.append(S.prim(S.AABB, mat, r.uniform(0.2, 1.0, 3), 0.2, list(c - h) + list(c + h)))
                else:
                    prims.append(S.sphere(c, float(r.uniform(0.8, 1.7)), mat, r.uniform(0.2, 1.0, 3), 0.2))
    w, h, spp, depth = 48, 32, 4, 8
    frm, at, vup = base, base + np.array([0.0, 0.0, 1.0]), np.array([0.0, 1.0, 0.0])
    sc = gpu.Scene.from_prims(prims)
    cam = gpu.camera_look(frm, at, vup, 70.0, 0.1, w, h)
    mean, u8, st = gpu.render(sc, cam, w, h, spp, depth, seed=5)
    omean, ou8, ocnt, _ = O.render(prims, O.camera_look(frm, at, vup, 70.0, 0.1, w, h), w, h, spp, depth,
                                   seed=5, threads=8)
    assert_parity(mean, u8, st, omean, ou8, ocnt)
    monkeypatch.setenv("FR_BVH", "0")
    mean0, _, st0 = gpu.render(gpu.Scene.from_prims(prims), cam, w, h, spp, depth, seed=5)
    assert np.array_equal(mean0.view(np.uint32), mean.view(np.uint32)) and st0["hits"] == st["hits"]


@pytest.mark.parametrize("aperture", [0.0, 0.1, 2e-30, 1e-33, 3.0])
def test_lens_radius_prescale_and_its_fallback(gpu, aperture):
    """camera.rs:62-66's lens offset: the trace kernel multiplies the accepted disk point's
    integers k by lens * 2^-23 when that product is exact (render.hip, KCam::lens_pre) and
    scales k by 2^-23 first otherwise (aperture 1e-33: lens * 2^-23 underflows); a zero, a
    tiny, the scenes' and a large aperture, both trace kernels, against the oracle bit for bit."""
    name, w, h, spp, depth = "scene_08", 48, 27, 4, 8
    sc = gpu.Scene.from_file(gpu.scene_path(name), w, h)
    prims, (frm, at, vup, fov) = S.load_json(open(gpu.scene_path(name)).read())
    cam = gpu.camera_look(frm, at, vup, fov, aperture, w, h)
    omean, ou8, ocnt, _ = O.render(prims, O.camera_look(frm, at, vup, fov, aperture, w, h), w, h, spp, depth,
                                   seed=7, threads=8)
    for jit in (False, "wait"):
        mean, u8, st = gpu.render(sc, cam, w, h, spp, depth, seed=7, scene_jit=jit)
        assert_parity(mean, u8, st, omean, ou8, ocnt)
        assert np.array_equal(mean.view(np.uint32), omean.view(np.uint32))


# ---- save_image_mt (tracer.rs:83-158) ---------------------------------------------

@pytest.mark.parametrize("which,w,h,sample", [(0, 32, 18, 3), (0, 40, 24, 1), (2, 36, 22, 20), (0, 16, 3, 2)])
def test_save_image_mt_bands_match_oracle(gpu, which, w, h, sample):
    """4 row bands of H/4 rows with the band offset in v, per-pass u8, u8 average; rows past
    4*(H/4) stay 0 (h = 3: no band rows at all)."""
    sc = gpu.Scene.builtin(which, w, h)
    acc, u8, st = gpu.render(sc, sc.camera, w, h, sample, 50, seed=0x5EED, mt_bands=True)
    oacc, ou8, ocnt = O.render_mt(S.BUILTIN[which](), O.camera_new(w, h), w, h, sample, 50, 0x5EED)
    assert np.array_equal(acc.view(np.uint32), oacc.view(np.uint32))
    assert np.array_equal(u8, ou8)
    assert (st["segments"], st["hits"]) == (ocnt["segments"], ocnt["hits"])
    assert not u8[4 * (h // 4):].any()


def test_save_image_mt_writes_png(gpu, tmp_path):
    m = gpu.create_model(24, 16)
    out = tmp_path / "basic_mt.png"
    acc, u8, st = gpu.save_image_mt(m, 2, str(out))
    assert out.read_bytes()[:8] == b"\x89PNG\r\n\x1a\n" and u8.shape == (16, 24, 3)


@pytest.mark.parametrize("colors", ["nonneg", "negative", "negzero"])
def test_absorbed_paths_skip_unwind_only_when_exact(gpu, colors):
    """An absorbed path's colour is +0 through finite non-negative attenuations; with a
    negative or -0 attenuation component the product's zero sign depends on the chain,
    so the unwind must run (sc.att_nonneg). Bits of the mean are compared."""
    w, h, spp, depth = 40, 24, 3, 4
    prims = random_scene(21)
    if colors == "negative":
        prims[1]["color"] = np.array([-0.5, 0.25, 0.75], np.float32)
    elif colors == "negzero":
        prims[1]["color"] = np.array([-0.0, 0.25, 0.75], np.float32)
    sc = gpu.Scene.from_prims(prims)
    mean, u8, st = gpu.render(sc, gpu.camera_new(w, h), w, h, spp, depth, seed=5)
    omean, ou8, ocnt, _ = O.render(prims, O.camera_new(w, h), w, h, spp, depth, seed=5, threads=8)
    assert_parity(mean, u8, st, omean, ou8, ocnt)
    assert np.array_equal(mean.view(np.uint32), omean.view(np.uint32))


@pytest.mark.parametrize("n,bright,diffuse", [(14, False, False), (14, False, True), (6, False, True),
                                              (15, False, False), (14, True, False)])
def test_absorbed_paths_in_both_record_formats(gpu, n, bright, diffuse, monkeypatch):
    """Absorbed paths (a depth cap of 3; metal rejections when not diffuse) in scenes of up
    to 15 primitives, one with an attenuation above 1: the 8-B records (4-bit winners) and
    the 12-B records (FR_DEFER=1) give the oracle's bits."""
    w, h, spp, depth = 48, 32, 5, 3
    prims = random_scene(40 + n, n)
    if diffuse:
        for q in prims:
            if q["material"] in (S.METAL, S.DIELECTRIC):
                q["material"] = S.LAMBERTIAN
    if bright:
        prims[0]["color"] = np.array([1.5, 0.5, 0.5], np.float32)
    sc = gpu.Scene.from_prims(prims)
    mean, u8, st = gpu.render(sc, gpu.camera_new(w, h), w, h, spp, depth, seed=9)
    omean, ou8, ocnt, _ = O.render(prims, O.camera_new(w, h), w, h, spp, depth, seed=9, threads=8)
    assert_parity(mean, u8, st, omean, ou8, ocnt)
    assert np.array_equal(mean.view(np.uint32), omean.view(np.uint32))
    monkeypatch.setenv("FR_DEFER", "1")
    m12, _, _ = gpu.render(sc, gpu.camera_new(w, h), w, h, spp, depth, seed=9)
    assert np.array_equal(mean.view(np.uint32), m12.view(np.uint32))


@pytest.mark.parametrize("pipe,buf_gb,jit", [("1", None, False), ("2", None, False), ("3", None, False),
                                            ("5", None, False), ("2", "0.0002", False), ("3", None, "wait"),
                                            ("2", "0.0002", "wait")])
def test_pass_pipeline_never_changes_results(gpu, pipe, buf_gb, jit, monkeypatch):
    """Passes on alternating streams with a double-buffered sample buffer (and, with a
    tiny FR_SAMPLE_BUFFER_GB, many passes reusing the two slots) give the same bits; jit:
    the passes run the scene-specialised kernel."""
    w, h, spp = 64, 40, 70  # 5 blocks, the last partial
    sc = gpu.Scene.from_file(gpu.scene_path("scene_08"), w, h)
    monkeypatch.setenv("FR_PIPELINE", "1")
    monkeypatch.delenv("FR_SAMPLE_BUFFER_GB", raising=False)
    ref = gpu.render(sc, sc.camera, w, h, spp, 8)
    monkeypatch.setenv("FR_PIPELINE", pipe)
    if buf_gb:
        monkeypatch.setenv("FR_SAMPLE_BUFFER_GB", buf_gb)
    mean, u8, st = gpu.render(sc, sc.camera, w, h, spp, 8, scene_jit=jit)
    assert np.array_equal(mean.view(np.uint32), ref[0].view(np.uint32)) and np.array_equal(u8, ref[1])
    assert (st["segments"], st["hits"]) == (ref[2]["segments"], ref[2]["hits"])


@pytest.mark.slow
@pytest.mark.parametrize("shard,buf_gb", [(0, "8"), (7, None)])
def test_c4_shards_on_row_subsets(gpu, shard, buf_gb, monkeypatch):
    """C4 (scene_08 3840x2160, 1024 spp, 8 bounces) as ranks 0 and 7 of 8 render it: every
    10th row of the shard (28 of shard 0's 272 rows, 27 of shard 7's 264), all 3,840 pixels
    each, against the oracle. Shard 0
    runs with an 8-GB sample buffer (passes of 21 of its 64 blocks), shard 7 in one pass."""
    if buf_gb:
        monkeypatch.setenv("FR_SAMPLE_BUFFER_GB", buf_gb)
    w, h, spp, depth = 3840, 2160, 1024, 8
    sc = gpu.Scene.from_file(gpu.scene_path("scene_08"), w, h)
    mean, u8, st = gpu.render(sc, sc.camera, w, h, spp, depth, shard_index=shard, shard_count=8)
    mine = [y for y in range(h) if (y // 8) % 8 == shard]
    assert st["samples"] == len(mine) * w * spp
    assert np.isnan(mean[[y for y in range(h) if (y // 8) % 8 != shard]]).all()  # other shards untouched
    prims, (frm, at, vup, fov) = S.load_json(open(gpu.scene_path("scene_08")).read())
    cam = O.camera_look(frm, at, vup, fov, 0.1, w, h)
    rows = mine[::10]
    assert len(rows) >= 27
    omean, ou8, _ = O.render_rows(prims, cam, w, h, spp, depth, rows, threads=oracle_threads(), chunk=9,
                                  progress=_progress(f"C4 shard {shard}"))
    assert_parity(mean, u8, st, omean, ou8, None, rows=rows)


@pytest.mark.slow
def test_c5_generator_scene_on_full_rows(gpu):
    """C5 (10k spheres, 1920x1080, 512 spp, 8 bounces, BVH path) against the oracle's
    brute-force list loop on 64 full rows spread over the image (every 17th row from 0),
    122,880 pixels, 62.9 M samples, and on every row at every 32nd pixel (64,800 pixels,
    33.2 M samples), so every region of the image's traversals is compared (about 300 s
    of oracle on the GPU box's 16 CPUs). The BVH's list-order ties and padded t_max
    (tracer.rs:195-200) must give the list loop's winner everywhere."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_scene", os.path.join(ROOT, "tools", "gen_scene.py"))
    gs = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gs)
    text = gs.dumps(gs.generator_scene(10000, "sphere"))
    w, h, spp, depth = 1920, 1080, 512, 8
    sc = gpu.Scene.from_json(text, w, h)
    mean, u8, st = gpu.render(sc, sc.camera, w, h, spp, depth)
    prims, (frm, at, vup, fov) = S.load_json(text)
    cam = O.camera_look(frm, at, vup, fov, 0.1, w, h)
    rows = list(range(0, 17 * 64, 17))
    assert len(rows) == 64
    omean, ou8, _ = O.render_rows(prims, cam, w, h, spp, depth, rows, threads=oracle_threads(), chunk=2,
                                  progress=_progress("C5"))
    assert_parity(mean, u8, st, omean, ou8, None, rows=rows)
    assert np.isfinite(mean).all()
    cmean, cu8, _ = O.render_rows(prims, cam, w, h, spp, depth, range(h), threads=oracle_threads(), col_step=32,
                                  chunk=36, progress=_progress("C5 every row, col_step 32"))
    assert_parity(mean[:, ::32], u8[:, ::32], None, cmean[:, ::32], cu8[:, ::32], None)
    assert np.array_equal(mean[:, ::32].view(np.uint32), cmean[:, ::32].view(np.uint32))


@pytest.mark.parametrize("depth", [8, 12])
def test_absorbed_path_through_infinite_attenuation_is_nan(gpu, depth):
    """A fuzzy metal whose colour has an infinite component: an absorbed path (terminal
    +0) behind it is 0 * inf = NaN in the recursion (tracer.rs:206-207), so no unwind
    may be skipped there. depth 8 runs the u16-stack kernel, 12 the u32 one."""
    w, h, spp = 24, 16, 4
    prims = [S.sphere([0.0, 0.0, -2.0], 0.9, S.METAL, [np.inf, 0.5, 0.5], 1.0),
             S.sphere([0.0, -100.9, -2.0], 100.0, S.LAMBERTIAN, [0.5, 0.5, 0.5], 0.0)]
    sc = gpu.Scene.from_prims(prims)
    cam = gpu.camera_new(w, h)
    mean, u8, st = gpu.render(sc, cam, w, h, spp, depth, seed=77)
    omean, ou8, ocnt, _ = O.render(prims, O.camera_new(w, h), w, h, spp, depth, seed=77, threads=8)
    assert np.isnan(omean).any(), "fixture must absorb some path behind the metal"
    assert _same_bits(mean, omean)
    assert np.array_equal(u8, ou8)
    assert (st["segments"], st["hits"]) == (ocnt["segments"], ocnt["hits"])


def test_bvh_depth_cap_chain_scene(gpu, monkeypatch):
    """Spheres at exponentially growing distances: binned SAH peels a few off per level,
    so the builder must switch to median splits to keep every internal node within the
    kBvhStack-entry traversal stack (bvh.h). Checked against the list-order loop and
    the oracle."""
    prims = []
    for k in range(700):
        x = 1.02 ** k - 1.0
        prims.append(S.sphere((x - 3.0, 0.3 * np.sin(k), -3.0 - 0.01 * k), 0.05 + 0.002 * (k % 7), k % 4,
                              (0.2 + 0.001 * k, 0.5, 0.7), 0.3))
    prims.append(S.sphere((0.0, -1000.5, -1.0), 1000.0, 0, (0.5, 0.5, 0.5), 0.0))
    w, h, spp, depth = 40, 24, 2, 8
    cam = gpu.camera_new(w, h)
    mean, u8, st = gpu.render(gpu.Scene.from_prims(prims), cam, w, h, spp, depth, seed=5)
    omean, ou8, ocnt, _ = O.render(prims, O.camera_new(w, h), w, h, spp, depth, seed=5, threads=8)
    assert_parity(mean, u8, st, omean, ou8, ocnt)
    monkeypatch.setenv("FR_BVH", "0")
    mean0, _, st0 = gpu.render(gpu.Scene.from_prims(prims), cam, w, h, spp, depth, seed=5)
    assert np.array_equal(mean0.view(np.uint32), mean.view(np.uint32)) and st0["hits"] == st["hits"]


def test_bvh_at_the_depth_cap_matches_list_loop(gpu, monkeypatch):
    """150k spheres: leaves grow past kBvhLeafMax and the deepest internal node sits at
    the traversal stack's limit (bvh.cpp). The BVH result must equal the list-order loop
    bit for bit (the oracle is too slow at this size; the loop is pinned to it above)."""
    r = np.random.default_rng(11)
    c = r.uniform(-40, 40, (150000, 3)) * np.array([1.0, 0.15, 1.0]) + np.array([0, 0, -45.0])
    rad = r.uniform(0.05, 0.3, 150000)
    mats = r.integers(0, 4, 150000)
    prims = [S.sphere(c[k], rad[k], int(mats[k]), (0.6, 0.5, 0.4), 0.2) for k in range(len(c))]
    w, h, spp, depth = 32, 18, 1, 8
    cam = gpu.camera_new(w, h)
    mean, u8, st = gpu.render(gpu.Scene.from_prims(prims), cam, w, h, spp, depth, seed=9)
    assert st["hits"] > 0
    monkeypatch.setenv("FR_BVH", "0")
    mean0, _, st0 = gpu.render(gpu.Scene.from_prims(prims), cam, w, h, spp, depth, seed=9)
    assert np.array_equal(mean0.view(np.uint32), mean.view(np.uint32)) and st0["hits"] == st["hits"]
