"""Frames in flight: K renders of shard 0 of N alternating between C render contexts (each
its own streams and buffers), no host wait between them; reports ms per frame over the K
frames against the one-context serial loop. python tools/pipe_frames.py N [K] [C] [stream]
With "stream" no context waits for its previous frame on the host either (bench.py's loop:
the streams order a context's frames), so the comparison is streamed 1 context vs C."""
import json
import os
import sys
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fo-rma_amd"))
import forma_rt as fr  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
k = int(sys.argv[2]) if len(sys.argv) > 2 else 20
nc = int(sys.argv[3]) if len(sys.argv) > 3 else 2
stream = len(sys.argv) > 4 and sys.argv[4] == "stream"
sc = fr.Scene.from_file(fr.scene_path("scene_08"), 1920, 1080)
p = fr.make_params(1920, 1080, 256, 8, shard_index=0, shard_count=n)
ctxs = [fr.RenderContext(0) for _ in range(nc)]
frames = [fr.PinnedFrame(1920, 1080) for _ in range(nc)]


def run(contexts):
    for c in contexts:
        c.render(sc, sc.camera, p)
        c.sync()
    t = time.perf_counter()
    for i in range(k):
        c = contexts[i % len(contexts)]
        if i >= len(contexts) and not stream:
            c.wait()
        c.render(sc, sc.camera, p)
        c.download_async(frames[i % len(contexts)])
    for c in contexts:
        c.wait()
    return (time.perf_counter() - t) / k * 1e3


serial = run(ctxs[:1])
piped = run(ctxs)
print(json.dumps({"shards": n, "frames": k, "contexts": nc, "serial_ms_per_frame": round(serial, 3),
                  "pipelined_ms_per_frame": round(piped, 3)}), flush=True)
