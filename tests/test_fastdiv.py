"""Host check of the invariant-divisor division the trace kernel uses to split a work
item into (sample block, pixel slot): render.hip `fastdiv` / `fastdiv_magic`
(Granlund-Montgomery, 32-bit, round-up magic with the add-and-shift fix-up). The kernel
divides the tile-block index (< 2^26) by n_tiles (1 .. 2^16); this restates the formula
in numpy u64 arithmetic and compares it with exact integer division."""
import numpy as np


def magic(d):
    l = (d - 1).bit_length()  # ceil(log2 d); 0 for d = 1
    m = ((1 << 32) * ((1 << l) - d)) // d + 1
    assert m < (1 << 32)
    return m, min(l, 1) | (max(l - 1, 0) << 1)


def fastdiv(x, m, shifts):
    x = x.astype(np.uint64)
    t = (x * np.uint64(m)) >> np.uint64(32)
    return (t + ((x - t) >> np.uint64(shifts & 1))) >> np.uint64(shifts >> 1)


def test_fastdiv_small_divisors_exhaustive_range():
    x = np.arange(0, 1 << 20, dtype=np.uint64)
    for d in range(1, 600):
        m, l = magic(d)
        assert np.array_equal(fastdiv(x, m, l), x // np.uint64(d)), d


def test_fastdiv_kernel_divisors_edges():
    rng = np.random.default_rng(7)
    edges = np.array([0, 1, 2, 63, 64, 65, (1 << 26) - 1, (1 << 31) - 1, (1 << 31), (1 << 32) - 1], dtype=np.uint64)
    # n_tiles of every image size up to 8K x 8K rows-of-8 tilings, plus random divisors
    ds = list(range(600, 5000, 7)) + [32400, 8100, 4050, 2025, 65535, 65536] + list(rng.integers(2, 1 << 20, 200))
    for d in ds:
        d = int(d)
        m, l = magic(d)
        x = np.concatenate([edges, rng.integers(0, 1 << 32, 4096, dtype=np.uint64),
                            np.arange(0, 4 * d, dtype=np.uint64)[: 1 << 16],
                            (np.arange(1, 256, dtype=np.uint64) * np.uint64(d))[:, None].repeat(3, 1).ravel()
                            + np.tile(np.array([-1, 0, 1], dtype=np.int64), 255).astype(np.uint64)])
        x = x[x < (1 << 32)]
        assert np.array_equal(fastdiv(x, m, l), x // np.uint64(d)), d
