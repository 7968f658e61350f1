"""A compiled C consumer of include/forma_rt.h (tests/c/abi_consumer.c).

gcc builds it against the header and links it to libforma_rt.so, as the Rust binding
of INTEGRATION.md would bind the library. Its _Static_asserts pin every field offset
that binding's #[repr(C)] structs assume; here its printed layout is also compared
with the ctypes mirror (forma_rt.py), and on a GPU its render through fr_ctx_* (pinned
host buffers, asynchronous gather) must equal the ctypes path bit for bit.
"""
import ctypes as C
import json
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
SRC = os.path.join(ROOT, "tests", "c", "abi_consumer.c")
LIBDIR = os.path.join(ROOT, "fo-rma_amd")


@pytest.fixture(scope="module")
def consumer(tmp_path_factory, fr):
    exe = str(tmp_path_factory.mktemp("c") / "abi_consumer")
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-O1", "-I", os.path.join(ROOT, "include"), SRC,
                    "-L", LIBDIR, "-lforma_rt", f"-Wl,-rpath,{LIBDIR}", "-o", exe], check=True)
    return exe


def test_c_layout_matches_ctypes_mirror(consumer, fr):
    out = subprocess.run([consumer, "layout"], check=True, capture_output=True, text=True).stdout
    lay = json.loads(out)
    assert lay["abi_version"] == fr.FR_ABI_VERSION
    for cname, cls in (("fr_prim", fr.FrPrim), ("fr_camera", fr.FrCamera), ("fr_params", fr.FrParams),
                       ("fr_stats", fr.FrStats)):
        names = [f for f, _ in cls._fields_]
        assert sorted(k.split(".")[1] for k in lay if k.startswith(cname + ".")) == sorted(names), cname
        for f in names:
            field = getattr(cls, f)
            assert lay[f"{cname}.{f}"] == [field.offset, field.size], (cname, f)
    assert lay["sizeof"] == [C.sizeof(fr.FrPrim), C.sizeof(fr.FrCamera), C.sizeof(fr.FrParams),
                             C.sizeof(fr.FrStats)]


@pytest.mark.gpu
def test_c_consumer_render_equals_ctypes_path(consumer, gpu, tmp_path):
    """scene_08 at 64x36, 4 spp, depth 8 through the C program's fr_ctx_* calls and through
    ctypes: identical f32 means, u8 image and path counters."""
    w, h, spp, depth = 64, 36, 4, 8
    out = tmp_path / "frame.bin"
    subprocess.run([consumer, "render", gpu.scene_path("scene_08"), str(w), str(h), str(spp), str(depth), str(out)],
                   check=True, timeout=120)
    raw = out.read_bytes()
    n = w * h * 3
    mean = np.frombuffer(raw, np.float32, n).reshape(h, w, 3)
    u8 = np.frombuffer(raw, np.uint8, n, offset=4 * n).reshape(h, w, 3)
    cnt = np.frombuffer(raw, np.uint64, 4, offset=5 * n)
    sc = gpu.Scene.from_file(gpu.scene_path("scene_08"), w, h)
    m2, u2, st = gpu.render(sc, sc.camera, w, h, spp, depth)
    assert np.array_equal(mean.view(np.uint32), m2.view(np.uint32))
    assert np.array_equal(u8, u2)
    assert list(cnt) == [st["segments"], st["hits"], st["samples"], st["scatters"]]


@pytest.mark.gpu
@pytest.mark.parametrize("devices", ["0,0", "0"])
def test_c_consumer_multi_device_model_equals_ctypes_path(consumer, gpu, tmp_path, devices):
    """INTEGRATION.md's exact create_model / save_image sequence from C: fr_mctx_create over
    DEVICES, fr_mctx_render with FR_FLAG_WRITE_U8 | FR_FLAG_SCENE_JIT, fr_mctx_sync,
    fr_mctx_frame, fr_mctx_free (tracer.rs:19-28, 160-187). Both of its frames (the first
    may run the compiled-in kernel while the scene kernel compiles; the second, after
    fr_jit_wait, runs the scene kernel on every shard) equal the ctypes fr_ctx render bit for
    bit, with the same counters."""
    w, h, spp, depth = 72, 44, 5, 8  # H % 8 != 0: a partial last strip
    out = tmp_path / "mframe.bin"
    subprocess.run([consumer, "mrender", gpu.scene_path("scene_08"), str(w), str(h), str(spp), str(depth), str(out),
                    devices], check=True, timeout=300)
    raw = out.read_bytes()
    n, nd = w * h * 3, len(devices.split(","))
    sc = gpu.Scene.from_file(gpu.scene_path("scene_08"), w, h)
    m2, u2, st = gpu.render(sc, sc.camera, w, h, spp, depth)
    frame_bytes = 5 * n + 32 + 4 * nd
    assert len(raw) == 2 * frame_bytes
    for k in range(2):
        o = k * frame_bytes
        mean = np.frombuffer(raw, np.float32, n, offset=o).reshape(h, w, 3)
        u8 = np.frombuffer(raw, np.uint8, n, offset=o + 4 * n).reshape(h, w, 3)
        cnt = np.frombuffer(raw, np.uint64, 4, offset=o + 5 * n)
        states = list(np.frombuffer(raw, np.int32, nd, offset=o + 5 * n + 32))
        assert np.array_equal(mean.view(np.uint32), m2.view(np.uint32)), k
        assert np.array_equal(u8, u2), k
        assert list(cnt) == [st["segments"], st["hits"], st["samples"], st["scatters"]], k
        if k == 1:
            assert states == [gpu.FR_JIT_USED] * nd, states
        else:
            assert all(s in (gpu.FR_JIT_USED, gpu.FR_JIT_PENDING) for s in states), states
