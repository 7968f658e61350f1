"""bench.py's frame loop for every rank of N, one shard at a time on one device: K frames of
shard k of N of the headline workload enqueued back to back on one context, each gathered
asynchronously into page-locked memory, one wait at the end; prints ms per frame and the
trace kernel's mean HIP-event time per launch for each k, then a summary with the min and
max over shards. The slowest shard bounds an N-GPU frame (bench.py reports the max over
ranks), so DESIGN.md §6's predicted efficiency at N uses the max.

    python tools/shard_stream.py N [K] [--shards k0,k1,...]

Default shards: all of 0..N-1. FR_FRAME_PIPE / FR_SCENE_JIT pass through (A/B knobs)."""
import json
import os
import sys
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fo-rma_amd"))
import forma_rt as fr  # noqa: E402

W, H, SPP, DEPTH = 1920, 1080, 256, 8


def stream_shard(sc, frame, n, k, frames, jit):
    p = fr.make_params(W, H, SPP, DEPTH, shard_index=k, shard_count=n, scene_jit=jit)
    ctx = fr.RenderContext(0)
    ctx.prepare(sc, sc.camera, p)
    for _ in range(2):
        ctx.render(sc, sc.camera, p)
        ctx.download_async(frame)
    ctx.wait()
    ctx.trace_log(True)
    t = time.perf_counter()
    for _ in range(frames):
        ctx.render(sc, sc.camera, p)
        ctx.download_async(frame)
    st = ctx.sync()
    ctx.wait()
    ms = (time.perf_counter() - t) / frames * 1e3
    launches = ctx.trace_log_read()
    ctx.trace_log(False)
    ctx.close()
    return {"shards": n, "shard": k, "frames": frames, "ms_per_frame": round(ms, 4),
            "trace_ms_per_launch": round(sum(launches) / max(1, len(launches)), 4),
            "trace_launches": st["trace_launches"], "samples": st["samples"], "segments": st["segments"],
            "pipe": os.environ.get("FR_FRAME_PIPE", ""), "occupancy": st["occupancy"]}


def main():
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    n = int(args[0]) if args else 8
    frames = int(args[1]) if len(args) > 1 else 20
    shards = list(range(n))
    for i, x in enumerate(sys.argv):
        if x == "--shards":
            shards = [int(v) for v in sys.argv[i + 1].split(",")]
    jit = os.environ.get("FR_SCENE_JIT") != "0"
    sc = fr.Scene.from_file(fr.scene_path("scene_08"), W, H)
    frame = fr.PinnedFrame(W, H)
    rows = []
    for k in shards:
        r = stream_shard(sc, frame, n, k, frames, jit)
        rows.append(r)
        print(json.dumps(r), flush=True)
    ms = [r["ms_per_frame"] for r in rows]
    worst = max(rows, key=lambda r: r["ms_per_frame"])
    print(json.dumps({"shards": n, "summary": True, "timed": [r["shard"] for r in rows],
                      "ms_per_frame_min": min(ms), "ms_per_frame_max": max(ms),
                      "slowest_shard": worst["shard"], "samples_total": sum(r["samples"] for r in rows)}),
          flush=True)
    frame.close()


if __name__ == "__main__":
    main()
