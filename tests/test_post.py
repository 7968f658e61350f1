"""Post-process effects (src/shaders/compute/*.wgsl chained as in
rendering/post_processor.rs:101-129): the HIP passes against oracle/post_ref.py, bit for
bit, plus oracle sanity checks that need no GPU."""
import ctypes as C

import numpy as np
import pytest

from oracle import post_ref as P


def _img(seed, h, w):
    return np.random.default_rng(seed).integers(0, 256, (h, w, 4), dtype=np.uint8)


# ---- oracle sanity (CPU) ----------------------------------------------------------

def test_oracle_identities():
    img = _img(0, 19, 23)
    img[..., 3] = 255
    assert np.array_equal(P.effect(img, P.NONE), img)
    assert np.array_equal(P.chain(img, [P.INVERT_COLOR, P.INVERT_COLOR]), img)
    sq = _img(1, 17, 17)
    assert np.array_equal(P.effect(sq, P.FLIP_AXIS), sq.transpose(1, 0, 2))
    px = P.effect(img, P.PIXELATE)
    assert (px[:8, :8] == img[0, 0]).all() and (px[16:, 16:] == img[16, 16]).all()
    gray = np.repeat(np.arange(0, 256, 16, dtype=np.uint8)[None, :, None], 4, 2)
    g = P.effect(gray, P.GRAYSCALE)
    assert np.abs(g[..., :3].astype(int) - gray[..., :3]).max() <= 1  # NTSC weights sum to 1
    il = P.effect(img, P.INTERLACE)
    assert not il[0::2, :, :3].any() and np.array_equal(il[1::2], img[1::2])
    an = P.effect(img, P.ANAGLYPH)
    assert not an[:, :10, 0].any() and not an[:, -10:, 2].any() and (an[..., 3] == 255).all()


def test_oracle_flip_axis_drops_stores_outside():
    img = _img(2, 5, 9)
    out = P.effect(img, P.FLIP_AXIS)
    assert np.array_equal(out[:5, :5], img[:5, :5].transpose(1, 0, 2)) and not out[:, 5:].any()


# ---- device (GPU) -------------------------------------------------------------------

@pytest.mark.gpu
@pytest.mark.parametrize("e", range(12))
@pytest.mark.parametrize("shape", [(36, 64), (33, 17), (8, 200)])
def test_each_effect_matches_oracle(gpu, e, shape):
    img = _img(100 + e, *shape)
    out = gpu.post_process(img, [e], time=3.25)
    assert np.array_equal(out, P.effect(img, e, 3.25)), P.NAMES[e]


@pytest.mark.gpu
@pytest.mark.parametrize("seed", range(5))
def test_effect_chains_match_oracle(gpu, seed):
    r = np.random.default_rng(seed)
    effects = [int(v) for v in r.integers(0, 12, int(r.integers(1, 6)))]
    img = _img(seed, 45, 70)
    t = float(r.uniform(0, 100))
    assert np.array_equal(gpu.post_process(img, effects, time=t), P.chain(img, effects, t))


@pytest.mark.gpu
def test_post_on_a_render_device_path(gpu):
    """A render's u8 output -> RGBA on the device -> effect chain in place (no host copy)."""
    import torch
    w, h = 48, 32
    sc = gpu.Scene.builtin(2, w, h)
    ctx = gpu.RenderContext(0)
    ctx.render(sc, sc.camera, gpu.make_params(w, h, 2, 8))
    ctx.sync()
    mean, u8 = ctx.download(w, h)
    d_mean, d_u8 = ctx.device_buffers()
    rgba = torch.empty((h, w, 4), dtype=torch.uint8, device="cuda")
    scratch = torch.empty_like(rgba)
    lib = gpu.lib()
    gpu.check(lib.fr_rgb_to_rgba_device(None, C.c_void_p(d_u8), C.c_void_p(rgba.data_ptr()), w * h))
    effects = [P.WAVE, P.PIXELATE, P.NOISE]
    arr = (C.c_int * 3)(*effects)
    gpu.check(lib.fr_post_process_device(None, arr, 3, 1.5, w, h, C.c_void_p(rgba.data_ptr()),
                                         C.c_void_p(scratch.data_ptr())))
    torch.cuda.synchronize()
    host_in = np.concatenate([u8, np.full((h, w, 1), 255, np.uint8)], -1)
    assert np.array_equal(rgba.cpu().numpy(), P.chain(host_in, effects, 1.5))


def test_unknown_effect_is_an_error(fr):
    with pytest.raises(fr.ForMaError):
        fr.post_process(np.zeros((4, 4, 4), np.uint8), [12])
