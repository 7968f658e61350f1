"""Tail analysis from an FR_DIAG FR_DIAG_TIMES file: per wave start/end stamps plus the
first drained claim (100 MHz s_memrealtime)."""
import sys
import numpy as np

raw = np.fromfile(sys.argv[1], dtype=np.uint64)
t = raw[: 2 * 65536].reshape(-1, 2)
dr = raw[2 * 65536: 3 * 65536]
n = int((t[:, 1] > 0).sum())
t, dr = t[:n].astype(np.float64), dr[:n]
t0 = t[:, 0].min()
s, e = (t[:, 0] - t0) / 100.0, (t[:, 1] - t0) / 100.0
ok = dr != np.uint64(2 ** 64 - 1)
d = (dr[ok].astype(np.float64) - t0) / 100.0
print(f"waves {n}, kernel {e.max()/1e3:.3f} ms; first drain {d.min()/1e3:.3f} ms, median drain {np.median(d)/1e3:.3f} ms")
tail = e[ok] - d
print(f"per-wave end - first drained claim: mean {tail.mean()/1e3:.3f} p50 {np.median(tail)/1e3:.3f} "
      f"p90 {np.percentile(tail, 90)/1e3:.3f} max {tail.max()/1e3:.3f} ms")
print(f"kernel end - first drain anywhere: {(e.max() - d.min())/1e3:.3f} ms")
# residency over time: fraction of the kernel's waves still running at each tenth
T = e.max()
for f in [0.5, 0.7, 0.8, 0.85, 0.9, 0.95, 0.98]:
    tt = f * T
    print(f"  t={tt/1e3:.3f} ms ({f:.0%}): {np.mean((s <= tt) & (e > tt)):.1%} of waves running")
print(f"  wave starts: first {s.min()/1e3:.4f} ms, last {s.max()/1e3:.4f} ms")
# iterations (appended after the drain stamps: per wave, end << 32 | at first drain)
if raw.size >= 4 * 65536:
    it = raw[3 * 65536: 4 * 65536][:n]
    i_end, i_dr = (it >> np.uint64(32)).astype(np.float64), (it & np.uint64(0xFFFFFFFF)).astype(np.float64)
    okk = ok & (i_end > 0)
    rate_all = e[okk] / np.maximum(i_end[okk], 1)
    rate_tail = (e[okk] - (dr[okk].astype(np.float64) - t0) / 100.0) / np.maximum(i_end[okk] - i_dr[okk], 1)
    print(f"iterations per wave: mean {i_end[okk].mean():.0f}; after first drain mean {(i_end - i_dr)[okk].mean():.0f} "
          f"max {(i_end - i_dr)[okk].max():.0f}")
    print(f"us per iteration: whole kernel mean {rate_all.mean():.2f}; after drain mean {rate_tail.mean():.2f} "
          f"p10 {np.percentile(rate_tail, 10):.2f} p90 {np.percentile(rate_tail, 90):.2f}")
    last = np.argsort(e[okk])[-5:]
    print("last 5 waves: end ms", np.round(e[okk][last] / 1e3, 3), "drain ms",
          np.round((dr[okk][last].astype(np.float64) - t0) / 1e5, 3), "iters after drain", (i_end - i_dr)[okk][last])
