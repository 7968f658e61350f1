"""bench.py's frame loop for one rank of N, on one device: K frames of shard 0 of N of the
headline workload enqueued back to back on one context, each gathered asynchronously into
page-locked memory, one wait at the end; prints ms per frame (A/B of FR_FRAME_PIPE and
FR_SCENE_JIT without the distributed launcher).  python tools/shard_stream.py N [K]"""
import json
import os
import sys
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fo-rma_amd"))
import forma_rt as fr  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
sc = fr.Scene.from_file(fr.scene_path("scene_08"), 1920, 1080)
p = fr.make_params(1920, 1080, 256, 8, shard_index=0, shard_count=n, scene_jit=os.environ.get("FR_SCENE_JIT") != "0")
ctx = fr.RenderContext(0)
frame = fr.PinnedFrame(1920, 1080)
ctx.prepare(sc, sc.camera, p)
for _ in range(2):
    ctx.render(sc, sc.camera, p)
    ctx.download_async(frame)
ctx.wait()
t = time.perf_counter()
for _ in range(k):
    ctx.render(sc, sc.camera, p)
    ctx.download_async(frame)
st = ctx.sync()
ctx.wait()
ms = (time.perf_counter() - t) / k * 1e3
print(json.dumps({"shards": n, "frames": k, "ms_per_frame": round(ms, 4), "pipe": os.environ.get("FR_FRAME_PIPE", ""),
                  "occupancy": st["occupancy"], "trace_ms": round(st["trace_ms"], 4)}), flush=True)
