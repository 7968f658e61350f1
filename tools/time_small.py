"""Time a small frame (BASELINE C1 by default) the way bench.py's config_c1 does: frames
streamed back to back into a page-locked frame, one sync at the end; prints ms per step and
the mean render time from the launch log.

    FORMA_RT_LIB=... python tools/time_small.py [scene W H SPP DEPTH STEPS]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(
    os.path.abspath(__file__)))), "fo-rma_amd"))
import forma_rt as fr  # noqa: E402

a = sys.argv[1:]
scene, w, h, spp, depth, steps = (a[0], *map(int, a[1:6])) if a else ("scene_01", 256, 256, 4, 4, 20)
sc = fr.Scene.from_file(fr.scene_path(scene), w, h)
ctx = fr.RenderContext(0)
p = fr.make_params(w, h, spp, depth)
frame = fr.PinnedFrame(w, h)
for _ in range(3):
    ctx.render(sc, sc.camera, p)
    ctx.download_async(frame)
ctx.wait()
has_log = hasattr(fr.lib(), "fr_ctx_trace_log") and os.environ.get("NO_LOG") != "1"
if has_log:
    ctx.trace_log(True)
t = time.perf_counter()
host_r = host_d = 0.0
for _ in range(steps):
    t1 = time.perf_counter()
    ctx.render(sc, sc.camera, p)
    t2 = time.perf_counter()
    ctx.download_async(frame)
    host_r += t2 - t1
    host_d += time.perf_counter() - t2
ctx.sync()
ctx.wait()
dt = (time.perf_counter() - t) / steps
out = {"scene": scene, "ms_per_step": round(dt * 1e3, 4), "host_render_call_ms": round(host_r / steps * 1e3, 4),
       "host_download_call_ms": round(host_d / steps * 1e3, 4)}
if has_log:
    fl = ctx.trace_log_read(frames=True)
    tl = ctx.trace_log_read()
    out["render_ms"] = round(sum(fl) / len(fl), 4)
    out["trace_ms"] = round(sum(tl) / len(tl), 4)
t = time.perf_counter()
for _ in range(steps):
    ctx.render(sc, sc.camera, p)
    ctx.sync()
out["sync_each_ms"] = round((time.perf_counter() - t) / steps * 1e3, 4)
print(json.dumps(out), flush=True)
