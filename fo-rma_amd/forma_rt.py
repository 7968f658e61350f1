"""Python host mirror of fo-rma's tracer API over libforma_rt's C ABI.

Same names, argument meaning and failure behaviour as the reference's operator
API in cpu_ray_tracer/tracer.rs (paths relative to the reference root):

    create_model(width, height)          tracer.rs:19-28
    update(model, keys, delta_time)      tracer.rs:30-55   (orbit camera + 1-spp frame)
    save_image(model, sample, path)      tracer.rs:160-187 (sample spp, PNG)
    TraceModel                           tracer.rs:12-17

and the Hitable plugin API (shapes/hitable.rs:4-14): Sphere / Plane / Box objects
with translate()/rotate(), flattened into the ordered primitive list the GPU
kernel consumes. Rendering always runs the HIP kernel: if libforma_rt.so or a
GPU is missing this module raises — there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import struct
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# FORMA_RT_LIB selects another build of the same ABI (used for A/B kernel variants)
LIB_PATH = os.environ.get("FORMA_RT_LIB") or os.path.join(HERE, "libforma_rt.so")
SCENES_DIR = os.path.join(HERE, "scenes")

FR_ABI_VERSION = 6  # include/forma_rt.h FR_ABI_VERSION
FR_OK, FR_EARG, FR_EPARSE, FR_EHIP, FR_ENODEV, FR_ENOMEM = 0, -1, -2, -3, -4, -5
FR_SPHERE, FR_PLANE, FR_AABB, FR_OBB, FR_STUB, FR_TRIANGLE = 0, 1, 2, 3, 4, 5
FR_LAMBERTIAN, FR_METAL, FR_DIELECTRIC, FR_LIGHT = 0, 1, 2, 3
FR_FLAG_WRITE_U8 = 1
FR_FLAG_MT_BANDS = 2  # save_image_mt semantics (forma_rt.h)
FR_FLAG_SCENE_JIT = 4  # scene-specialised trace kernel (hiprtc, cached; same image bits)
FR_FLAG_SCENE_JIT_WAIT = 8  # ... compiled on the render's thread when missing (else in the background)
FR_FLAG_SCENE_JIT_CACHED = 16  # ... only when already built or on disk; never compiled (one-shot callers)
FR_JIT_OFF, FR_JIT_USED, FR_JIT_PENDING, FR_JIT_FAILED, FR_JIT_MISS = 0, 1, 2, 3, 4  # fr_ctx_jit_state
MAX_DEPTH = 50  # tracer.rs:10
DEFAULT_SEED = 0x5EED


class ForMaError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"libforma_rt error {code}: {msg}")
        self.code = code


class FrPrim(C.Structure):
    _fields_ = [("kind", C.c_uint32), ("material", C.c_uint32), ("color", C.c_float * 3), ("fuzz", C.c_float),
                ("g", C.c_float * 16)]


class FrCamera(C.Structure):
    _fields_ = [(n, C.c_float * 3) for n in ("position", "lower_left", "horizontal", "vertical", "u", "v", "w")] + [
        (n, C.c_float) for n in ("aspect", "lens_radius", "focus_dist", "radius", "rotation")]

    def to_array(self):
        vals = []
        for n in ("position", "lower_left", "horizontal", "vertical", "u", "v", "w"):
            vals.extend(getattr(self, n))
        vals += [self.aspect, self.lens_radius, self.focus_dist, self.radius, self.rotation]
        return np.asarray(vals, dtype=np.float32)


class FrParams(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("spp", C.c_uint32), ("max_depth", C.c_uint32),
                ("seed", C.c_uint64), ("strip_rows", C.c_uint32), ("shard_index", C.c_uint32),
                ("shard_count", C.c_uint32), ("flags", C.c_uint32)]


class FrStats(C.Structure):
    _fields_ = [("segments", C.c_uint64), ("hits", C.c_uint64), ("samples", C.c_uint64), ("prim_tests", C.c_uint64),
                ("kernel_ms", C.c_double), ("total_ms", C.c_double), ("trace_ms", C.c_double),
                ("trace_launches", C.c_uint32), ("occupancy", C.c_uint32), ("scatters", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


# Every symbol include/forma_rt.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "fr_last_error", "fr_abi_version", "fr_device_count",
    "fr_scene_create", "fr_scene_builtin", "fr_scene_from_json", "fr_scene_free", "fr_scene_count",
    "fr_scene_get_prims", "fr_scene_translate", "fr_scene_rotate",
    "fr_camera_init", "fr_camera_look", "fr_camera_orbit", "fr_camera_translate", "fr_update_delta",
    "fr_ctx_create", "fr_ctx_free", "fr_ctx_render", "fr_ctx_sync", "fr_ctx_download", "fr_ctx_download_async",
    "fr_ctx_wait", "fr_ctx_device_buffers", "fr_host_alloc", "fr_host_free", "fr_ctx_trace_log",
    "fr_ctx_trace_log_read", "fr_mctx_create", "fr_mctx_free", "fr_mctx_count", "fr_mctx_ctx", "fr_mctx_render",
    "fr_mctx_sync", "fr_mctx_frame", "fr_mctx_download",
    "fr_render_hip", "fr_render_hip_multi", "fr_selftest_ops", "fr_selftest_rng", "fr_selftest_recip",
    "fr_selftest_div",
    "fr_post_process", "fr_post_process_device", "fr_rgb_to_rgba_device", "fr_ctx_jit_info", "fr_selftest_jit",
    "fr_ctx_prepare", "fr_ctx_jit_state", "fr_jit_wait",
)

_lib = None


def _load_torch_runtime_first():
    # If torch is importable, load it first so this library binds the same
    # libamdhip64 (soname libamdhip64.so.7) as torch: one HIP runtime per process.
    # FR_NO_TORCH=1 skips it (a short-lived profiled child that never imports torch).
    if os.environ.get("FR_NO_TORCH") == "1":
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib():
    """Load libforma_rt.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ForMaError(FR_ENODEV, f"{LIB_PATH} not built; run __graft_entry__.build() or make -C fo-rma_amd")
    _load_torch_runtime_first()
    L = C.CDLL(LIB_PATH)
    P = C.POINTER
    vp = C.c_void_p
    f3 = P(C.c_float)
    L.fr_last_error.restype = C.c_char_p
    L.fr_abi_version.restype = C.c_int
    L.fr_device_count.argtypes = [P(C.c_int)]
    L.fr_scene_create.argtypes = [P(FrPrim), C.c_uint32, P(vp)]
    L.fr_scene_builtin.argtypes = [C.c_int, C.c_uint32, C.c_uint32, P(vp), P(FrCamera)]
    L.fr_scene_from_json.argtypes = [C.c_char_p, C.c_size_t, C.c_uint32, C.c_uint32, P(vp), P(FrCamera)]
    L.fr_scene_free.argtypes = [vp]
    L.fr_scene_free.restype = None
    L.fr_scene_count.argtypes = [vp]
    L.fr_scene_count.restype = C.c_uint32
    L.fr_scene_get_prims.argtypes = [vp, P(FrPrim), C.c_uint32]
    L.fr_scene_translate.argtypes = [vp, C.c_uint32, f3]
    L.fr_scene_rotate.argtypes = [vp, C.c_uint32, f3]
    L.fr_camera_init.argtypes = [P(FrCamera), C.c_uint32, C.c_uint32]
    L.fr_camera_look.argtypes = [P(FrCamera), f3, f3, f3, C.c_float, C.c_float, C.c_uint32, C.c_uint32]
    L.fr_camera_orbit.argtypes = [P(FrCamera), f3]
    L.fr_camera_translate.argtypes = [P(FrCamera), f3]
    L.fr_update_delta.argtypes = [C.c_uint8, C.c_float, f3]
    L.fr_ctx_create.argtypes = [C.c_int, vp, P(vp)]
    L.fr_ctx_free.argtypes = [vp]
    L.fr_ctx_free.restype = None
    L.fr_ctx_render.argtypes = [vp, vp, P(FrCamera), P(FrParams)]
    L.fr_ctx_sync.argtypes = [vp, P(FrStats)]
    L.fr_ctx_download.argtypes = [vp, f3, P(C.c_uint8)]
    L.fr_ctx_device_buffers.argtypes = [vp, P(vp), P(vp)]
    if hasattr(L, "fr_ctx_download_async"):  # absent from A/B builds of older sources
        L.fr_ctx_download_async.argtypes = [vp, f3, P(C.c_uint8)]
        L.fr_ctx_wait.argtypes = [vp]
        L.fr_host_alloc.argtypes = [C.c_size_t, P(vp)]
        L.fr_host_free.argtypes = [vp]
        L.fr_host_free.restype = None
    if hasattr(L, "fr_mctx_create"):  # absent from A/B builds of older sources
        L.fr_ctx_trace_log.argtypes = [vp, C.c_int]
        L.fr_ctx_trace_log_read.argtypes = [vp, C.c_int, P(C.c_double), C.c_uint32, P(C.c_uint32)]
        L.fr_mctx_create.argtypes = [P(C.c_int), C.c_int, P(vp)]
        L.fr_mctx_free.argtypes = [vp]
        L.fr_mctx_free.restype = None
        L.fr_mctx_count.argtypes = [vp]
        L.fr_mctx_ctx.argtypes = [vp, C.c_int, P(vp)]
        L.fr_mctx_render.argtypes = [vp, vp, P(FrCamera), P(FrParams)]
        L.fr_mctx_sync.argtypes = [vp, P(FrStats)]
        L.fr_mctx_frame.argtypes = [vp, P(P(C.c_float)), P(P(C.c_uint8))]
        L.fr_mctx_download.argtypes = [vp, f3, P(C.c_uint8)]
    L.fr_render_hip.argtypes = [vp, P(FrCamera), P(FrParams), C.c_int, f3, P(C.c_uint8), P(FrStats)]
    L.fr_render_hip_multi.argtypes = [vp, P(FrCamera), P(FrParams), C.c_int, f3, P(C.c_uint8), P(FrStats)]
    L.fr_selftest_ops.argtypes = [C.c_int, C.c_int, f3, f3, C.c_uint32, f3]
    L.fr_selftest_rng.argtypes = [C.c_int, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, P(C.c_uint32)]
    if hasattr(L, "fr_post_process"):  # absent from A/B builds of older sources
        L.fr_post_process.argtypes = [C.c_int, P(C.c_int), C.c_uint32, C.c_float, C.c_uint32, C.c_uint32,
                                      P(C.c_uint8), P(C.c_uint8)]
        L.fr_post_process_device.argtypes = [vp, P(C.c_int), C.c_uint32, C.c_float, C.c_uint32, C.c_uint32, vp, vp]
        L.fr_rgb_to_rgba_device.argtypes = [vp, vp, vp, C.c_size_t]
    if hasattr(L, "fr_selftest_recip"):  # absent from A/B builds of older sources
        L.fr_selftest_recip.argtypes = [C.c_int, C.c_uint64, C.c_uint64, P(C.c_uint64), P(C.c_uint32)]
    if hasattr(L, "fr_selftest_div"):  # absent from A/B builds of older sources
        L.fr_selftest_div.argtypes = [C.c_int, C.c_uint32, C.c_uint32, P(C.c_uint64), P(C.c_uint64)]
    if hasattr(L, "fr_ctx_jit_info"):  # absent from A/B builds of older sources
        L.fr_ctx_jit_info.argtypes = [vp, P(C.c_int), P(C.c_double), P(C.c_int)]
        L.fr_ctx_prepare.argtypes = [vp, vp, P(FrCamera), P(FrParams)]
    if hasattr(L, "fr_ctx_jit_state"):  # absent from A/B builds of older sources
        L.fr_ctx_jit_state.argtypes = [vp, P(C.c_int)]
        L.fr_jit_wait.argtypes = []
        L.fr_selftest_jit.argtypes = [C.c_char_p, P(C.c_uint32), C.c_uint32, P(C.c_int), P(C.c_size_t), P(C.c_double)]
    _lib = L
    return L


def check(rc):
    if rc != FR_OK:
        raise ForMaError(rc, lib().fr_last_error().decode(errors="replace"))
    return rc


def _f3(v):
    return (C.c_float * 3)(*[float(np.float32(x)) for x in v])


def device_count():
    n = C.c_int(0)
    rc = lib().fr_device_count(C.byref(n))
    return n.value if rc == FR_OK else 0


# ---- Hitable plugin objects (shapes/hitable.rs:4-14) ------------------------

class Hitable:
    """Base of the tracer's shapes. translate/rotate are no-ops unless a shape
    overrides them (hitable.rs:12-13)."""
    kind = FR_STUB

    def __init__(self, material=0, color=(0.0, 0.0, 0.0), fuzz=0.0):
        self.material, self.color, self.fuzz = int(material), tuple(color), float(fuzz)

    def geometry(self):
        return ()

    def translate(self, v):
        pass

    def rotate(self, v):
        pass

    def to_prim(self):
        p = FrPrim()
        p.kind, p.material, p.fuzz = self.kind, self.material, self.fuzz
        for i in range(3):
            p.color[i] = self.color[i]
        for i, g in enumerate(self.geometry()):
            p.g[i] = g
        return p


class Sphere(Hitable):
    """shapes/sphere.rs: Sphere::new(center, radius, material, color, fuzz)"""
    kind = FR_SPHERE

    def __init__(self, center, radius, material, color, fuzz):
        super().__init__(material, color, fuzz)
        self.center, self.radius = tuple(center), float(radius)

    def geometry(self):
        return tuple(self.center) + (self.radius,)


class Plane(Hitable):
    """shapes/plane.rs: Plane::new(position, orientation, size, material, color, fuzz)"""
    kind = FR_PLANE

    def __init__(self, position, orientation, size, material, color, fuzz):
        super().__init__(material, color, fuzz)
        self.position, self.orientation, self.size = tuple(position), tuple(orientation), tuple(size)

    def geometry(self):
        return tuple(self.position) + tuple(self.orientation) + tuple(self.size)

    def translate(self, v):  # plane.rs:62-64
        self.position = tuple(v)

    def rotate(self, v):  # plane.rs:66-68
        self.orientation = tuple(v)


class Box(Hitable):
    """The build's axis-aligned box (FR_AABB), given by min/max corners."""
    kind = FR_AABB

    def __init__(self, mn, mx, material, color, fuzz):
        super().__init__(material, color, fuzz)
        self.mn, self.mx = tuple(mn), tuple(mx)

    def geometry(self):
        return tuple(self.mn) + tuple(self.mx)


class Triangle(Hitable):
    """The build's triangle (FR_TRIANGLE), vertices v0, v1, v2 in winding order."""
    kind = FR_TRIANGLE

    def __init__(self, v0, v1, v2, material, color, fuzz):
        super().__init__(material, color, fuzz)
        self.v = (tuple(v0), tuple(v1), tuple(v2))

    def geometry(self):
        return self.v[0] + self.v[1] + self.v[2]


class Stub(Hitable):
    """shapes/aabb.rs / rectangle.rs: never hit, never scatter."""
    kind = FR_STUB


# ---- scenes and cameras -----------------------------------------------------

class Scene:
    """An ordered primitive list on the host plus its resident device copies
    (cpu_ray_tracer/scene.rs:4-7)."""

    def __init__(self, handle, camera=None):
        self._h = C.c_void_p(handle) if not isinstance(handle, C.c_void_p) else handle
        self.camera = camera

    @classmethod
    def from_objects(cls, objects, camera=None):
        arr = (FrPrim * max(1, len(objects)))(*[o.to_prim() for o in objects])
        h = C.c_void_p()
        check(lib().fr_scene_create(arr, len(objects), C.byref(h)))
        return cls(h, camera)

    @classmethod
    def from_prims(cls, prims, camera=None):
        """prims: sequence of FrPrim (or dicts with kind/material/color/fuzz/g)"""
        arr = (FrPrim * max(1, len(prims)))()
        for i, p in enumerate(prims):
            if isinstance(p, FrPrim):
                arr[i] = p
            else:
                arr[i].kind, arr[i].material, arr[i].fuzz = p["kind"], p["material"], float(p["fuzz"])
                for k in range(3):
                    arr[i].color[k] = float(p["color"][k])
                for k in range(16):
                    arr[i].g[k] = float(p["g"][k])
        h = C.c_void_p()
        check(lib().fr_scene_create(arr, len(prims), C.byref(h)))
        return cls(h, camera)

    @classmethod
    def builtin(cls, which, width, height):
        """0 get_simple_scene, 1 get_plane_scene, 2 get_objects (scenes.rs), 3 simple
        scene in the interactive frontend's state. Camera = Camera::new(w, h)."""
        h, cam = C.c_void_p(), FrCamera()
        check(lib().fr_scene_builtin(which, width, height, C.byref(h), C.byref(cam)))
        return cls(h, cam)

    @classmethod
    def from_json(cls, text, width, height):
        if isinstance(text, str):
            text = text.encode()
        h, cam = C.c_void_p(), FrCamera()
        check(lib().fr_scene_from_json(text, len(text), width, height, C.byref(h), C.byref(cam)))
        return cls(h, cam)

    @classmethod
    def from_file(cls, path, width, height):
        with open(path, "rb") as f:
            return cls.from_json(f.read(), width, height)

    def __len__(self):
        return lib().fr_scene_count(self._h)

    def prims(self):
        n = len(self)
        arr = (FrPrim * max(1, n))()
        check(lib().fr_scene_get_prims(self._h, arr, n))
        return [arr[i] for i in range(n)]

    def translate(self, index, v):
        check(lib().fr_scene_translate(self._h, index, _f3(v)))

    def rotate(self, index, v):
        check(lib().fr_scene_rotate(self._h, index, _f3(v)))

    def close(self):
        if self._h and self._h.value:
            lib().fr_scene_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def camera_new(width, height):
    cam = FrCamera()
    check(lib().fr_camera_init(C.byref(cam), width, height))
    return cam


def camera_look(frm, at, vup, fov, aperture, width, height):
    cam = FrCamera()
    check(lib().fr_camera_look(C.byref(cam), _f3(frm), _f3(at), _f3(vup), float(fov), float(aperture), width,
                               height))
    return cam


def camera_orbit(cam, delta):
    check(lib().fr_camera_orbit(C.byref(cam), _f3(delta)))
    return cam


def camera_translate(cam, delta):
    check(lib().fr_camera_translate(C.byref(cam), _f3(delta)))
    return cam


def scene_path(name):
    """Path of a bundled scene file (the reference's scenes/*.json, re-serialised)."""
    return os.path.join(SCENES_DIR, f"{name}.min.json")


# ---- rendering ----------------------------------------------------------------

def make_params(width, height, spp, max_depth=MAX_DEPTH, seed=DEFAULT_SEED, shard_index=0, shard_count=1,
                write_u8=True, mt_bands=False, scene_jit=False):
    """scene_jit: False, True (the scene kernel once it is compiled; until then renders run
    the compiled-in kernel, same bits), "wait" (compile on the render's thread if needed) or
    "cached" (the scene kernel only if already built or on disk; never a compile)."""
    p = FrParams()
    p.width, p.height, p.spp, p.max_depth, p.seed = width, height, spp, max_depth, seed
    p.strip_rows, p.shard_index, p.shard_count = 8, shard_index, shard_count
    p.flags = ((FR_FLAG_WRITE_U8 if write_u8 else 0) | (FR_FLAG_MT_BANDS if mt_bands else 0) |
               (FR_FLAG_SCENE_JIT if scene_jit else 0) | (FR_FLAG_SCENE_JIT_WAIT if scene_jit == "wait" else 0) |
               (FR_FLAG_SCENE_JIT_CACHED if scene_jit == "cached" else 0))
    return p


def jit_wait():
    """Block until no scene-kernel compile is queued or running in this process."""
    check(lib().fr_jit_wait())


class _PinnedBlock:
    """One fr_host_alloc allocation. Freed when the last reference goes: every numpy view
    made by _pinned_views holds one (through its ctypes buffer), so an array a caller kept
    never points at freed memory."""

    def __init__(self, nbytes):
        self.ptr = C.c_void_p()
        check(lib().fr_host_alloc(max(1, nbytes), C.byref(self.ptr)))
        self.nbytes = nbytes

    def __del__(self):
        try:
            if self.ptr and self.ptr.value:
                lib().fr_host_free(self.ptr)
                self.ptr = C.c_void_p()
        except Exception:
            pass


def _pinned_views(block, width, height):
    n = width * height * 3
    buf = (C.c_uint8 * block.nbytes).from_address(block.ptr.value)
    buf._owner = block  # the buffer (the arrays' base) keeps the allocation alive
    mean = np.frombuffer(buf, dtype=np.float32, count=n).reshape(height, width, 3)
    u8 = np.frombuffer(buf, dtype=np.uint8, count=n, offset=n * 4).reshape(height, width, 3)
    return mean, u8


class PinnedFrame:
    """Full-image host buffers in page-locked memory (fr_host_alloc): mean [H, W, 3] f32
    and u8 [H, W, 3], the targets of RenderContext.download_async. close() drops the
    frame's own views; the memory is returned once no view of it is left anywhere."""

    def __init__(self, width, height):
        self.width, self.height = width, height
        self._block = _PinnedBlock(width * height * 3 * 5)
        self.mean, self.u8 = _pinned_views(self._block, width, height)

    def close(self):
        self.mean = self.u8 = None
        self._block = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class RenderContext:
    """One device, one HIP stream, resident output buffers (fr_ctx)."""

    def __init__(self, device=0, stream=None):
        self._h = C.c_void_p()
        check(lib().fr_ctx_create(device, C.c_void_p(stream) if stream else None, C.byref(self._h)))
        self.device = device

    def render(self, scene, cam, params):
        check(lib().fr_ctx_render(self._h, scene._h, C.byref(cam), C.byref(params)))

    def sync(self):
        st = FrStats()
        check(lib().fr_ctx_sync(self._h, C.byref(st)))
        return st.as_dict()

    def download(self, width, height, mean=None, u8=None):
        mean = np.full((height, width, 3), np.nan, dtype=np.float32) if mean is None else mean
        u8 = np.zeros((height, width, 3), dtype=np.uint8) if u8 is None else u8
        check(lib().fr_ctx_download(self._h, mean.ctypes.data_as(C.POINTER(C.c_float)),
                                    u8.ctypes.data_as(C.POINTER(C.c_uint8))))
        return mean, u8

    def download_into(self, mean=None, u8=None):
        """Copy the last render's strips into caller-owned full-image arrays (either may be
        None: that output is not copied). Page-locked arrays (PinnedFrame) copy by DMA."""
        fp = None if mean is None else mean.ctypes.data_as(C.POINTER(C.c_float))
        up = None if u8 is None else u8.ctypes.data_as(C.POINTER(C.c_uint8))
        check(lib().fr_ctx_download(self._h, fp, up))

    def download_async(self, frame):
        """Enqueue the last render's D2H gather into `frame` (a PinnedFrame); returns at
        once. The copies finish before wait() returns and before the next render writes
        its outputs; the next render's trace kernel overlaps them."""
        check(lib().fr_ctx_download_async(self._h, frame.mean.ctypes.data_as(C.POINTER(C.c_float)),
                                          frame.u8.ctypes.data_as(C.POINTER(C.c_uint8))))

    def wait(self):
        """Block until every render and download enqueued on this context has finished."""
        check(lib().fr_ctx_wait(self._h))

    def prepare(self, scene, cam, params):
        """Set up everything a render of `params` needs (scene copy, buffers, and with
        scene_jit the scene-specialised kernel) without rendering; returns jit_info()."""
        check(lib().fr_ctx_prepare(self._h, scene._h, C.byref(cam), C.byref(params)))
        return self.jit_info()

    def jit_info(self):
        """The last render's trace kernel: {"used": scene-specialised kernel ran, "ms": time
        that render spent getting it (compile or cache load), "compiled": hiprtc ran}."""
        used, ms, comp = C.c_int(0), C.c_double(0.0), C.c_int(0)
        check(lib().fr_ctx_jit_info(self._h, C.byref(used), C.byref(ms), C.byref(comp)))
        return {"used": bool(used.value), "ms": ms.value, "compiled": bool(comp.value), "state": self.jit_state()}

    def jit_state(self):
        """FR_JIT_OFF / USED / PENDING / FAILED for the last render (fr_ctx_jit_state)."""
        s = C.c_int(0)
        check(lib().fr_ctx_jit_state(self._h, C.byref(s)))
        return s.value

    def trace_log(self, enable=True):
        """Start (or stop) logging every trace-kernel launch's HIP-event duration."""
        check(lib().fr_ctx_trace_log(self._h, 1 if enable else 0))

    def trace_log_read(self, frames=False, timeline=False):
        """HIP-event durations (ms) logged since trace_log(True): every trace-kernel launch,
        or (frames=True) every whole render (trace + sum kernels). timeline=True: (start, end)
        pairs instead, in ms from the first logged trace launch's start."""
        which = (1 if frames else 0) + (2 if timeline else 0)
        n = C.c_uint32(0)
        check(lib().fr_ctx_trace_log_read(self._h, which, None, 0, C.byref(n)))
        k = 2 if timeline else 1
        arr = (C.c_double * max(1, k * n.value))()
        check(lib().fr_ctx_trace_log_read(self._h, which, arr, k * n.value, C.byref(n)))
        if timeline:
            return [(arr[2 * i], arr[2 * i + 1]) for i in range(n.value)]
        return [arr[i] for i in range(n.value)]

    def device_buffers(self):
        """(d_mean_rgb, d_rgb8) device addresses of the last render's full-image outputs."""
        dm, du = C.c_void_p(), C.c_void_p()
        check(lib().fr_ctx_device_buffers(self._h, C.byref(dm), C.byref(du)))
        return dm.value, du.value

    def close(self):
        if getattr(self, "_borrowed", False):
            return
        if self._h and self._h.value:
            lib().fr_ctx_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MultiContext:
    """fr_mctx: one fr_ctx per entry of `devices` (entries may repeat), shard i of n of
    every frame on entry i, the strips gathered asynchronously into one page-locked host
    frame. Persistent: frames of the same size allocate nothing (tracer.rs:83-134's row
    tiling, one device per shard instead of one thread)."""

    def __init__(self, devices):
        devs = (C.c_int * len(devices))(*[int(d) for d in devices])
        self._h = C.c_void_p()
        check(lib().fr_mctx_create(devs, len(devices), C.byref(self._h)))
        self.devices = list(devices)
        self._shape = None

    def render(self, scene, cam, params):
        """Enqueue one frame (all shards and their gathers); returns at once."""
        check(lib().fr_mctx_render(self._h, scene._h, C.byref(cam), C.byref(params)))
        self._shape = (params.height, params.width, 3)

    def sync(self):
        st = FrStats()
        check(lib().fr_mctx_sync(self._h, C.byref(st)))
        return st.as_dict()

    def frame(self):
        """(mean, u8) numpy copies of the host frame of the last render (after sync)."""
        fp, up = C.POINTER(C.c_float)(), C.POINTER(C.c_uint8)()
        check(lib().fr_mctx_frame(self._h, C.byref(fp), C.byref(up)))
        n = self._shape[0] * self._shape[1] * 3
        mean = np.ctypeslib.as_array(fp, shape=(n,)).reshape(self._shape).copy()
        u8 = np.ctypeslib.as_array(up, shape=(n,)).reshape(self._shape).copy()
        return mean, u8

    def frame_ptrs(self):
        """Host addresses of the page-locked frame (mean, u8)."""
        fp, up = C.POINTER(C.c_float)(), C.POINTER(C.c_uint8)()
        check(lib().fr_mctx_frame(self._h, C.byref(fp), C.byref(up)))
        return C.cast(fp, C.c_void_p).value, C.cast(up, C.c_void_p).value

    def context(self, i):
        """The i-th shard's RenderContext view (not owned: do not close it)."""
        h = C.c_void_p()
        check(lib().fr_mctx_ctx(self._h, i, C.byref(h)))
        rc = RenderContext.__new__(RenderContext)
        rc._h, rc.device, rc._borrowed = h, self.devices[i], True
        return rc

    def close(self):
        if self._h and self._h.value:
            lib().fr_mctx_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def render(scene, cam, width, height, spp, max_depth=MAX_DEPTH, seed=DEFAULT_SEED, device=0, shard_index=0,
           shard_count=1, n_gpus=1, mt_bands=False, scene_jit=False):
    """Render on the GPU. Returns (mean[H,W,3] f32, u8[H,W,3], stats). Rows outside the
    shard are NaN / 0. n_gpus > 1 row-shards the whole image across devices 0..n-1.
    mt_bands: save_image_mt semantics (mean then holds the u8 average, 0..255).
    scene_jit: the scene-specialised trace kernel (FR_FLAG_SCENE_JIT; same bits)."""
    mean = np.full((height, width, 3), np.nan, dtype=np.float32)
    u8 = np.zeros((height, width, 3), dtype=np.uint8)
    st = FrStats()
    p = make_params(width, height, spp, max_depth, seed, shard_index, shard_count, mt_bands=mt_bands,
                    scene_jit=scene_jit)
    fm, fu = mean.ctypes.data_as(C.POINTER(C.c_float)), u8.ctypes.data_as(C.POINTER(C.c_uint8))
    if n_gpus > 1:
        check(lib().fr_render_hip_multi(scene._h, C.byref(cam), C.byref(p), n_gpus, fm, fu, C.byref(st)))
    else:
        check(lib().fr_render_hip(scene._h, C.byref(cam), C.byref(p), device, fm, fu, C.byref(st)))
    return mean, u8, st.as_dict()


# ---- post-process effects (src/shaders/compute/*.wgsl) -------------------------

EFFECTS = ["none", "noise", "pixelate", "invert_color", "wave", "interlace", "flipaxis", "grayscale", "step",
           "watercolor", "chromostereopsis", "anaglyph"]  # shader_utils.rs:58-88 order and names


def post_process(rgba, effects, time=0.0, device=0):
    """Run the effect chain (post_processor.rs:101-129) on an [H, W, 4] uint8 image (or an
    [H, W, 3] one, given alpha 255). `effects`: ids or names. Returns a new [H, W, 4] array."""
    img = np.ascontiguousarray(rgba, dtype=np.uint8)
    if img.shape[-1] == 3:
        img = np.concatenate([img, np.full(img.shape[:2] + (1,), 255, np.uint8)], -1)
    ids = [EFFECTS.index(e) if isinstance(e, str) else int(e) for e in effects]
    h, w, _ = img.shape
    out = np.empty_like(img)
    arr = (C.c_int * max(1, len(ids)))(*ids)
    check(lib().fr_post_process(device, arr, len(ids), float(time), w, h,
                                img.ctypes.data_as(C.POINTER(C.c_uint8)), out.ctypes.data_as(C.POINTER(C.c_uint8))))
    return out


# ---- tracer.rs operator API ---------------------------------------------------

class TraceModel:
    """tracer.rs:12-17 {scene, width, height, pixels}, plus the render context the frames
    run on: one fr_ctx per model, created on the first frame and reused by every later
    update() / save_image() (no per-frame stream, event or buffer allocation)."""

    def __init__(self, scene, width, height):
        self.scene, self.width, self.height = scene, width, height
        self.pixels = np.zeros(width * height * 3, dtype=np.uint8)
        self.frame = 0
        self.seed = DEFAULT_SEED
        self.device = 0
        self.ctx = None
        self.last_stats = None
        self._pinned = None  # page-locked home of `pixels` once update() runs on the device

    def context(self):
        if self.ctx is None:
            self.ctx = RenderContext(self.device)
        return self.ctx

    def render(self, scene, spp, max_depth, seed, mt_bands=False, scene_jit=False):
        """One frame on the model's context: (mean[H,W,3], u8[H,W,3], stats). scene_jit: the
        trace kernel compiled for the scene once ready (same bits; compiled in the background,
        so a render never waits for it)."""
        ctx = self.context()
        ctx.render(scene, self.scene.camera, make_params(self.width, self.height, spp, max_depth, seed,
                                                         mt_bands=mt_bands, scene_jit=scene_jit))
        self.last_stats = ctx.sync()
        mean, u8 = ctx.download(self.width, self.height)
        return mean, u8, self.last_stats

    def frame_u8(self, scene, max_depth, seed):
        """update()'s frame: 1 spp, only the u8 image copied back, by DMA into page-locked
        memory that `pixels` views (overwritten by the next frame, as tracer.rs's
        model.pixels is). The view keeps the page-locked block alive, so an array returned
        here stays valid memory after the model is closed or collected; copy it to keep a
        frame past the next update()."""
        ctx = self.context()
        ctx.render(scene, self.scene.camera, make_params(self.width, self.height, 1, max_depth, seed))
        self.last_stats = ctx.sync()
        if self._pinned is None:
            self._pinned = PinnedFrame(self.width, self.height)
        ctx.download_into(u8=self._pinned.u8)
        self.pixels = self._pinned.u8.reshape(-1)
        return self.pixels

    def close(self):
        if self._pinned is not None:
            # model.pixels (and any array update() returned) keeps the page-locked block
            # alive by itself; only the model's own frame object goes
            self._pinned.close()
            self._pinned = None
        if self.ctx is not None:
            self.ctx.close()
            self.ctx = None


def create_model(width, height, scene=None):
    """tracer.rs:19-28: Scene::new = get_simple_scene + Camera::new(w, h)."""
    if scene is None:
        scene = Scene.builtin(0, width, height)
    elif scene.camera is None:
        scene.camera = camera_new(width, height)
    return TraceModel(scene, width, height)


def update(model, keys, delta_time, max_depth=MAX_DEPTH):
    """tracer.rs:30-55: key bitmask 00EQADWS -> camera.orbit(delta), then one 1-spp frame
    into model.pixels. Each frame draws from its own RNG key."""
    d = (C.c_float * 3)()
    check(lib().fr_update_delta(int(keys) & 0xFF, float(delta_time), d))
    camera_orbit(model.scene.camera, list(d))
    seed = model.seed ^ (0x9E3779B97F4A7C15 * (model.frame + 1) & 0xFFFFFFFFFFFFFFFF)
    model.frame += 1
    return model.frame_u8(model.scene, max_depth, seed)


def write_png(path, rgb8):
    """Minimal RGB8 PNG writer (the reference uses the image crate, tracer.rs:186)."""
    h, w, _ = rgb8.shape
    raw = b"".join(b"\x00" + rgb8[y].tobytes() for y in range(h))

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n")
        f.write(chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)))
        f.write(chunk(b"IDAT", zlib.compress(raw, 6)))
        f.write(chunk(b"IEND", b""))


def save_image_mt(model, sample, path="out/basic_mt.png", max_depth=MAX_DEPTH):
    """tracer.rs:136-158: `sample` passes of render_mt (4 row bands over the plain simple
    scene, scenes::get_simple_scene, with the model's camera), each pass gamma-corrected
    to u8, the u8 frames averaged and truncated, PNG."""
    simple = Scene.builtin(0, model.width, model.height)
    # a one-shot call: the scene kernel if it is cached, never a compile (which a process that
    # exits after this call would wait for at exit)
    acc, u8, stats = model.render(simple, sample, max_depth, model.seed, mt_bands=True, scene_jit="cached")
    write_png(path, u8)
    return acc, u8, stats


def save_image(model, sample, path="out/basic.png", max_depth=MAX_DEPTH):
    """tracer.rs:160-187: `sample` spp per pixel, gamma 2, u8, PNG. Like the reference it
    fails if the output directory is missing (tracer.rs:186 unwrap)."""
    mean, u8, stats = model.render(model.scene, sample, max_depth, model.seed, scene_jit="cached")
    write_png(path, u8)
    return mean, u8, stats
