"""bench.py's frame loop for every rank of N, one shard at a time on one device: K frames of
shard k of N of the headline workload enqueued back to back on one context, each gathered
asynchronously into page-locked memory, one wait at the end; prints ms per frame and the
trace kernel's mean HIP-event time per launch for each k, then a summary with the min and
max over shards. The slowest shard bounds an N-GPU frame (bench.py reports the max over
ranks), so DESIGN.md §6's predicted efficiency at N uses the max.

    python tools/shard_stream.py N [K] [--shards k0,k1,...] [--orders fwd,rev,shuf] [--warm W]

Default shards: all of 0..N-1. FR_FRAME_PIPE / FR_SCENE_JIT pass through (A/B knobs).
--orders runs the shard list once per order (fwd: as given, rev: reversed, shuf: a fixed
shuffle) and ends with a table of each shard's time over the orders and of each run
position's time over the orders: a slow shard that stays slow in every order is the shard's
work; a slow first (or last) position whatever the shard is the box or the run order."""
import json
import os
import random
import statistics
import sys
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fo-rma_amd"))
import forma_rt as fr  # noqa: E402

W, H, SPP, DEPTH = 1920, 1080, 256, 8


def stream_shard(sc, frame, n, k, frames, jit, warm=2):
    p = fr.make_params(W, H, SPP, DEPTH, shard_index=k, shard_count=n, scene_jit=jit)
    ctx = fr.RenderContext(0)
    ctx.prepare(sc, sc.camera, p)
    for _ in range(warm):
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
            "hits": st["hits"], "scatters": st["scatters"],
            "pipe": os.environ.get("FR_FRAME_PIPE", ""), "occupancy": st["occupancy"]}


def main():
    args = [x for x in sys.argv[1:] if not x.startswith("--")]
    n = int(args[0]) if args else 8
    frames = int(args[1]) if len(args) > 1 else 20
    shards = list(range(n))
    orders = ["fwd"]
    warm = 2
    for i, x in enumerate(sys.argv):
        if x == "--warm":
            warm = int(sys.argv[i + 1])
        if x == "--shards":
            shards = [int(v) for v in sys.argv[i + 1].split(",")]
        if x == "--orders":
            orders = sys.argv[i + 1].split(",")
    jit = os.environ.get("FR_SCENE_JIT") != "0"
    sc = fr.Scene.from_file(fr.scene_path("scene_08"), W, H)
    frame = fr.PinnedFrame(W, H)
    by_shard, by_pos = {}, {}
    for order in orders:
        seq = list(shards)
        if order == "rev":
            seq.reverse()
        elif order == "shuf":
            random.Random(12345).shuffle(seq)
        rows = []
        for pos, k in enumerate(seq):
            r = stream_shard(sc, frame, n, k, frames, jit, warm)
            r["order"], r["position"] = order, pos
            rows.append(r)
            by_shard.setdefault(k, []).append(r["ms_per_frame"])
            by_pos.setdefault(pos, []).append(r["ms_per_frame"])
            print(json.dumps(r), flush=True)
        ms = [r["ms_per_frame"] for r in rows]
        worst = max(rows, key=lambda r: r["ms_per_frame"])
        print(json.dumps({"shards": n, "summary": True, "order": order, "timed": [r["shard"] for r in rows],
                          "ms_per_frame_min": min(ms), "ms_per_frame_max": max(ms),
                          "slowest_shard": worst["shard"], "samples_total": sum(r["samples"] for r in rows)}),
              flush=True)
    if len(orders) > 1:
        med = lambda v: round(statistics.median(v), 4)  # noqa: E731
        print(json.dumps({"shards": n, "orders": orders,
                          "shard_median_ms": {k: med(v) for k, v in sorted(by_shard.items())},
                          "shard_ms": {k: v for k, v in sorted(by_shard.items())},
                          "position_median_ms": {p: med(v) for p, v in sorted(by_pos.items())}}), flush=True)
    frame.close()


if __name__ == "__main__":
    main()
