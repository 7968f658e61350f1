"""The C-ABI library loads and exports exactly what include/forma_rt.h declares."""
import ctypes as C
import os
import re

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
HEADER = os.path.join(ROOT, "include", "forma_rt.h")


def declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(fr_[a-z0-9_]+)\s*\(", text)))


def test_every_declared_symbol_is_exported(fr):
    names = declared()
    assert len(names) >= 25
    L = fr.lib()
    for n in names:
        assert hasattr(L, n), n
    assert sorted(fr.EXPORTS) == names


def test_abi_version_and_struct_sizes(fr):
    assert fr.lib().fr_abi_version() == fr.FR_ABI_VERSION == 6
    assert C.sizeof(fr.FrPrim) == 88
    assert C.sizeof(fr.FrCamera) == 26 * 4
    assert C.sizeof(fr.FrParams) == 40  # static_assert-ed in render.hip
    assert C.sizeof(fr.FrStats) == 72


def test_library_links_the_gfx950_code_object():
    data = open(os.path.join(ROOT, "fo-rma_amd", "libforma_rt.so"), "rb").read()
    assert b"gfx950" in data and b"trace_kernel" in data


def test_last_error_is_set_on_failure(fr):
    rc = fr.lib().fr_scene_builtin(42, 8, 8, C.byref(C.c_void_p()), None)
    assert rc == fr.FR_EARG
    assert b"unknown scene 42" in fr.lib().fr_last_error()


def test_render_without_device_fails_loudly(fr):
    if fr.device_count() > 0:
        return  # covered by the gpu tests on a GPU box
    sc = fr.Scene.builtin(0, 8, 8)
    try:
        fr.render(sc, sc.camera, 8, 8, 1)
    except fr.ForMaError as e:
        assert e.code in (fr.FR_ENODEV, fr.FR_EHIP)
    else:
        raise AssertionError("render returned without a GPU")


def test_header_abi_version_matches_host_mirror(fr):
    hdr = open(HEADER).read()
    m = re.search(r"#define FR_ABI_VERSION (\d+)", hdr)
    assert m and int(m.group(1)) == fr.FR_ABI_VERSION == fr.lib().fr_abi_version()
