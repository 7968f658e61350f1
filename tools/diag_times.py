"""Residency over time from an FR_DIAG run (FR_DIAG_TIMES file of per-wave
s_memrealtime start/end stamps, 100 MHz): how much of the kernel the wave slots
are busy, and how long the tail is."""
import sys

import numpy as np

t = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 2)
n = int(sys.argv[2]) if len(sys.argv) > 2 else int((t[:, 1] > 0).sum())
t = t[:n].astype(np.float64) / 100.0  # microseconds
t0 = t[:, 0].min()
s, e = t[:, 0] - t0, t[:, 1] - t0
dur = e.max()
grid = np.linspace(0, dur, 400)
active = np.array([((s <= g) & (e > g)).sum() for g in grid])
print(f"waves {n}, kernel {dur/1e3:.3f} ms, wave time mean {np.mean(e-s)/1e3:.3f} ms, "
      f"p50 {np.median(e-s)/1e3:.3f} max {np.max(e-s)/1e3:.3f} ms")
cap = active.max()
print(f"peak resident {cap}, mean resident {active.mean():.0f} ({active.mean()/cap:.1%} of peak)")
for frac in (0.99, 0.9, 0.75, 0.5):
    idx = np.where(active >= frac * cap)[0]
    print(f"  time with >= {frac:.0%} of peak resident: {len(idx)/len(grid):.1%}")
last_start = s.max()
print(f"last wave starts at {last_start/1e3:.3f} ms; tail after it {(dur-last_start)/1e3:.3f} ms")
