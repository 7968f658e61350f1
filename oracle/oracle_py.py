"""ctypes front-end of the oracle (TEST INFRASTRUCTURE ONLY).

Loads oracle/liboracle.so, the CPU restatement in oracle.cpp. Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg use this module.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


class OrCamera(C.Structure):
    _fields_ = [(n, C.c_float * 3) for n in ("position", "lower_left", "horizontal", "vertical", "u", "v", "w")] + [
        (n, C.c_float) for n in ("aspect", "lens_radius", "focus_dist", "radius", "rotation")]


class OrPrim(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("material", C.c_uint32), ("color", C.c_float * 3), ("fuzz", C.c_float),
                ("g", C.c_float * 16)]


class OrCounters(C.Structure):
    _fields_ = [("segments", C.c_uint64), ("hits", C.c_uint64), ("samples", C.c_uint64), ("scatters", C.c_uint64)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle` (or __graft_entry__.build())")
        L = C.CDLL(LIB_PATH)
        f3 = C.POINTER(C.c_float)
        L.oracle_camera_look.argtypes = [f3, f3, f3, C.c_float, C.c_float, C.c_uint32, C.c_uint32,
                                         C.POINTER(OrCamera)]
        L.oracle_camera_new.argtypes = [C.c_uint32, C.c_uint32, C.POINTER(OrCamera)]
        L.oracle_camera_orbit.argtypes = [C.POINTER(OrCamera), f3]
        L.oracle_camera_translate.argtypes = [C.POINTER(OrCamera), f3]
        L.oracle_rng_stream.argtypes = [C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.POINTER(C.c_uint32)]
        L.oracle_vec3.argtypes = [C.c_int, f3, f3, f3]
        L.oracle_refract.argtypes = [f3, f3, C.c_float, f3]
        L.oracle_refract.restype = C.c_int
        L.oracle_closest_hit.argtypes = [C.POINTER(OrPrim), C.c_uint32, f3, f3, f3]
        L.oracle_closest_hit.restype = C.c_int
        L.oracle_render.argtypes = [C.POINTER(OrPrim), C.c_uint32, C.POINTER(OrCamera), C.c_uint32, C.c_uint32,
                                    C.c_uint32, C.c_uint32, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32,
                                    C.c_uint32, C.c_int, f3, C.POINTER(C.c_uint8), C.POINTER(OrCounters)]
        L.oracle_render.restype = C.c_int64
        L.oracle_render_rows.argtypes = [C.POINTER(OrPrim), C.c_uint32, C.POINTER(OrCamera), C.c_uint32, C.c_uint32,
                                         C.c_uint32, C.c_uint32, C.c_uint64, C.POINTER(C.c_uint32), C.c_uint32,
                                         C.c_uint32, C.c_int, f3, C.POINTER(C.c_uint8), C.POINTER(OrCounters)]
        L.oracle_render_rows.restype = C.c_int64
        _lib = L
    return _lib


def _fa(v):
    return (C.c_float * 3)(*[float(np.float32(x)) for x in v])


def prims_to_c(prims):
    arr = (OrPrim * max(1, len(prims)))()
    for i, p in enumerate(prims):
        arr[i].kind = p["kind"]
        arr[i].material = p["material"]
        for k in range(3):
            arr[i].color[k] = float(p["color"][k])
        arr[i].fuzz = float(p["fuzz"])
        for k in range(16):
            arr[i].g[k] = float(p["g"][k])
    return arr


def camera_new(width, height):
    c = OrCamera()
    lib().oracle_camera_new(width, height, C.byref(c))
    return c


def camera_look(frm, at, vup, fov, aperture, width, height):
    c = OrCamera()
    lib().oracle_camera_look(_fa(frm), _fa(at), _fa(vup), float(fov), float(aperture), width, height, C.byref(c))
    return c


def camera_orbit(cam, delta):
    lib().oracle_camera_orbit(C.byref(cam), _fa(delta))
    return cam


def camera_translate(cam, delta):
    lib().oracle_camera_translate(C.byref(cam), _fa(delta))
    return cam


def camera_to_array(cam):
    """all 26 f32 camera fields in camera.rs order"""
    vals = []
    for n in ("position", "lower_left", "horizontal", "vertical", "u", "v", "w"):
        vals.extend(getattr(cam, n))
    vals += [cam.aspect, cam.lens_radius, cam.focus_dist, cam.radius, cam.rotation]
    return np.asarray(vals, dtype=np.float32)


def rng_stream(seed, pixel, sample, n):
    out = (C.c_uint32 * n)()
    lib().oracle_rng_stream(seed, pixel, sample, n, out)
    return np.frombuffer(out, dtype=np.uint32).copy()


def vec3(op, a, b=(0.0, 0.0, 0.0)):
    out = (C.c_float * 3)()
    lib().oracle_vec3(op, _fa(a), _fa(b), out)
    return np.frombuffer(out, dtype=np.float32).copy()


def refract(v, n, ni):
    out = (C.c_float * 3)()
    ok = lib().oracle_refract(_fa(v), _fa(n), float(ni), out)
    return bool(ok), np.frombuffer(out, dtype=np.float32).copy()


def closest_hit(prims, o, d):
    rec = (C.c_float * 7)()
    best = lib().oracle_closest_hit(prims_to_c(prims), len(prims), _fa(o), _fa(d), rec)
    return best, np.frombuffer(rec, dtype=np.float32).copy()


def render(prims, cam, width, height, spp, max_depth, seed=0x5EED, shard_index=0, shard_count=1, row_step=1,
           threads=1, col_step=1):
    """save_image semantics over a row subset (every col_step-th pixel of those rows);
    returns (mean[H,W,3] f32 (NaN where not rendered), u8[H,W,3], counters dict, rows
    rendered)"""
    mean = np.full((height, width, 3), np.nan, dtype=np.float32)
    u8 = np.zeros((height, width, 3), dtype=np.uint8)
    cnt = OrCounters()
    rows = lib().oracle_render(prims_to_c(prims), len(prims), C.byref(cam), width, height, spp, max_depth, seed,
                               shard_index, shard_count, row_step, col_step, threads,
                               mean.ctypes.data_as(C.POINTER(C.c_float)),
                               u8.ctypes.data_as(C.POINTER(C.c_uint8)), C.byref(cnt))
    if rows < 0:
        raise ValueError("oracle_render: bad arguments")
    return mean, u8, {"segments": cnt.segments, "hits": cnt.hits, "samples": cnt.samples,
                      "scatters": cnt.scatters}, int(rows)


def render_rows(prims, cam, width, height, spp, max_depth, rows, seed=0x5EED, threads=1, col_step=1, chunk=None,
                progress=None, out=None):
    """save_image semantics on an explicit list of image rows, rendered `chunk` rows per
    oracle call (progress(done, total) after each). out=(mean, u8, counters) continues
    filling earlier results. Returns (mean, u8, counters dict)."""
    if out is None:
        mean = np.full((height, width, 3), np.nan, dtype=np.float32)
        u8 = np.zeros((height, width, 3), dtype=np.uint8)
        tot = {"segments": 0, "hits": 0, "samples": 0, "scatters": 0}
    else:
        mean, u8, tot = out
    rows = [int(r) for r in rows]
    chunk = chunk or max(1, len(rows))
    pc = prims_to_c(prims)
    for i in range(0, len(rows), chunk):
        part = rows[i:i + chunk]
        arr = (C.c_uint32 * len(part))(*part)
        cnt = OrCounters()
        r = lib().oracle_render_rows(pc, len(prims), C.byref(cam), width, height, spp, max_depth, seed, arr, len(part),
                                     col_step, threads, mean.ctypes.data_as(C.POINTER(C.c_float)),
                                     u8.ctypes.data_as(C.POINTER(C.c_uint8)), C.byref(cnt))
        if r < 0:
            raise ValueError("oracle_render_rows: bad arguments")
        for k in tot:
            tot[k] += getattr(cnt, k)
        if progress:
            progress(min(i + chunk, len(rows)), len(rows))
    return mean, u8, tot


def render_mt(prims, cam, width, height, sample, max_depth=50, seed=0x5EED):
    """save_image_mt semantics (tracer.rs:136-158): returns (acc[H,W,3] f32, u8[H,W,3], counters)."""
    L = lib()
    if not getattr(L.oracle_render_mt, "argtypes", None):
        L.oracle_render_mt.argtypes = [C.POINTER(OrPrim), C.c_uint32, C.POINTER(OrCamera), C.c_uint32, C.c_uint32,
                                       C.c_uint32,
                                       C.c_uint32, C.c_uint64, C.POINTER(C.c_float), C.POINTER(C.c_uint8),
                                       C.POINTER(OrCounters)]
    acc = np.zeros((height, width, 3), dtype=np.float32)
    u8 = np.zeros((height, width, 3), dtype=np.uint8)
    cnt = OrCounters()
    rc = L.oracle_render_mt(prims_to_c(prims), len(prims), C.byref(cam),
                            width, height, sample, max_depth, seed, acc.ctypes.data_as(C.POINTER(C.c_float)),
                            u8.ctypes.data_as(C.POINTER(C.c_uint8)), C.byref(cnt))
    if rc != 0:
        raise ValueError("oracle_render_mt: bad arguments")
    return acc, u8, {"segments": cnt.segments, "hits": cnt.hits, "samples": cnt.samples, "scatters": cnt.scatters}
