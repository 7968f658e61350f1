"""Post-process effects oracle (TEST INFRASTRUCTURE ONLY).

A numpy float32 restatement of the 12 compute shaders in src/shaders/compute/*.wgsl
and their chaining in rendering/post_processor.rs:101-129, with the build's choices for
what WGSL leaves to the implementation: u8 -> f32 is u / 255,
f32 -> u8 is rint(clamp(x, 0, 1) * 255) (half to even), loads outside the image read 0,
stores outside it are dropped and a pass's destination starts cleared, and every f32
expression is evaluated as written, left to right, without contraction. Effect ids
follow shader_utils.rs:58-71. Nothing here is imported by the product.
"""
import numpy as np

F = np.float32
NONE, NOISE, PIXELATE, INVERT_COLOR, WAVE, INTERLACE, FLIP_AXIS, GRAYSCALE, STEP, WATERCOLOR, \
    CHROMOSTEREOPSIS, ANAGLYPH = range(12)
NAMES = ["none", "noise", "pixelate", "invert_color", "wave", "interlace", "flipaxis", "grayscale", "step",
         "watercolor", "chromostereopsis", "anaglyph"]


def _load(img):
    return img.astype(F) / F(255.0)


def _store(c):
    c = np.where(np.isnan(c), F(0.0), c)
    return np.rint(np.clip(c, F(0.0), F(1.0)) * F(255.0)).astype(np.uint8)


def _fract(v):
    return (v - np.floor(v)).astype(F)


def _luma(c):
    return (c[..., 0] * F(0.299) + c[..., 1] * F(0.587)) + c[..., 2] * F(0.114)


def _hash_wc(px, py):  # watercolor.comp.wgsl:7-10
    ax, ay, az = _fract(F(px) * F(0.1031)), _fract(F(py) * F(0.1031)), _fract(F(px) * F(0.1031))
    d = (ax * (ay + F(33.333)) + ay * (az + F(33.333))) + az * (ax + F(33.333))
    return _fract((ax + ay) * d)


def _hash_noise(x, y, time):  # noise.comp.wgsl:28-33
    fx, fy = x.astype(F) / F(10.0), y.astype(F) / F(10.0)
    t = F(time) * F(0.05)
    vx, vy = fx * F(0.3183099) + t, fy * F(0.3678794) + t
    return _fract(F(23.0) * _fract((vx * vy) * (vx + vy)))


def effect(img, e, time=0.0):
    """One shader pass over an [H, W, 4] uint8 image; returns the new image."""
    h, w, _ = img.shape
    c = _load(img)
    y, x = np.mgrid[0:h, 0:w]
    out = np.zeros_like(img)
    one = np.ones((h, w), F)
    if e == NONE:
        o = c
    elif e == NOISE:
        n = _hash_noise(x, y, time) / F(20.0)
        o = np.stack([c[..., 0] + n, c[..., 1] + n, c[..., 2] + n, one], -1)
    elif e == PIXELATE:
        o = c[(y // 8) * 8, (x // 8) * 8]
    elif e == INVERT_COLOR:
        o = np.stack([F(1.0) - c[..., 0], F(1.0) - c[..., 1], F(1.0) - c[..., 2], one], -1)
    elif e == WAVE:
        l = _luma(c)
        o = np.stack([l, l, l, one], -1)
        r = np.stack([one, c[..., 1], F(0.1) * c[..., 2], one], -1)
        o = np.where((c[..., 0] > F(0.4))[..., None], r, o)
        g = np.stack([F(0.1) * one, c[..., 1], F(0.1) * c[..., 2], one], -1)
        o = np.where((c[..., 1] > F(0.4))[..., None], g, o)
        b = np.stack([F(0.1) * c[..., 0], c[..., 1], one, one], -1)
        o = np.where((c[..., 2] > F(0.4))[..., None], b, o)
    elif e == INTERLACE:
        f = np.where(y % 2 == 0, F(0.0), F(1.0)).astype(F)
        o = np.stack([c[..., 0] * f, c[..., 1] * f, c[..., 2] * f, c[..., 3]], -1)
    elif e == FLIP_AXIS:  # stored at (y, x); stores outside the image are dropped
        keep = (y < w) & (x < h)
        out[x[keep], y[keep]] = _store(c[keep])
        return out
    elif e == GRAYSCALE:
        l = _luma(c)
        o = np.stack([l, l, l, c[..., 3]], -1)
    elif e == STEP:
        b = np.floor(_luma(c) / F(0.2)).astype(F) * F(0.2)
        o = np.stack([b, b, b, c[..., 3]], -1)
    elif e == WATERCOLOR:
        o = c.copy()
        px, py = x.astype(F), y.astype(F)
        qw, qh = F(w) / F(4.0), F(h) / F(4.0)
        for i in range(50):
            fi = F(i)
            csx, csy = fi * F(123.45), F(67.89)
            cx = qw + (_hash_wc(csx, csy) * qw) * F(2.0)
            cy = qh + (_hash_wc(csx + F(1.0), csy) * qh) * F(2.0)
            radius = F(10.0) + _hash_wc(fi * F(234.56), F(78.9)) * F(200.0)
            r = _hash_wc(fi * F(345.67), F(89.01))
            dx, dy = px - cx, py - cy
            inside = np.sqrt(dx * dx + dy * dy) <= radius
            o[..., 0] = np.where(inside, o[..., 0] + r * F(0.05), o[..., 0])
            o[..., 1] = np.where(inside, o[..., 1] + F(0.0) * F(0.05), o[..., 1])
            o[..., 2] = np.where(inside, o[..., 2] + F(0.0) * F(0.05), o[..., 2])
            o[..., 3] = np.where(inside, o[..., 3] + F(1.0) * F(0.05), o[..., 3])
    elif e == CHROMOSTEREOPSIS:
        r = np.where(c[..., 0] - c[..., 2] > F(0.0), F(1.0), F(0.0)).astype(F)
        o = np.stack([r, np.zeros_like(r), F(1.0) - r, one], -1)
    elif e == ANAGLYPH:
        def at(xx, ch):
            ok = (xx >= 0) & (xx < w)
            return np.where(ok, c[y, np.clip(xx, 0, w - 1), ch], F(0.0))
        o = np.stack([at(x - 10, 0), np.zeros((h, w), F), at(x + 10, 2), one], -1)
    else:
        raise ValueError(e)
    return _store(o.astype(F))


def chain(img, effects, time=0.0):
    for e in effects:
        img = effect(img, e, time)
    return img
