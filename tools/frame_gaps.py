"""Timeline of bench.py's streamed frame loop without a profiler: the HIP events the library
logs around every trace launch and every render (fr_ctx_trace_log, which 2 / 3), so the
time between one trace's end and the next one's start (the frame's cost beyond its trace)
is seen directly.

    python tools/frame_gaps.py [K] [--no-download] [--shard k/n]

--shard k/n: shard k of n of the frame (one rank of n GPUs); its traces may overlap (two
trace streams), so gaps can be negative."""
import json
import os
import statistics
import sys
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fo-rma_amd"))
import forma_rt as fr  # noqa: E402

W, H, SPP, DEPTH = 1920, 1080, 256, 8


def main():
    k = int(sys.argv[1]) if len(sys.argv) > 1 and not sys.argv[1].startswith("--") else 20
    download = "--no-download" not in sys.argv
    k_sh, n_sh = 0, 1
    for i, a in enumerate(sys.argv):
        if a == "--shard":
            k_sh, n_sh = map(int, sys.argv[i + 1].split("/"))
    sc = fr.Scene.from_file(fr.scene_path("scene_08"), W, H)
    p = fr.make_params(W, H, SPP, DEPTH, shard_index=k_sh, shard_count=n_sh, scene_jit=True)
    frame = fr.PinnedFrame(W, H)
    ctx = fr.RenderContext(0)
    ctx.prepare(sc, sc.camera, p)
    for _ in range(2):
        ctx.render(sc, sc.camera, p)
        if download:
            ctx.download_async(frame)
    ctx.wait()
    ctx.trace_log(True)
    t = time.perf_counter()
    for _ in range(k):
        ctx.render(sc, sc.camera, p)
        if download:
            ctx.download_async(frame)
    ctx.sync()
    ctx.wait()
    wall = (time.perf_counter() - t) / k * 1e3
    tr = ctx.trace_log_read(timeline=True)
    rd = ctx.trace_log_read(frames=True, timeline=True)
    ctx.close()
    frame.close()
    gaps = [tr[i + 1][0] - tr[i][1] for i in range(len(tr) - 1)]
    period = [tr[i + 1][0] - tr[i][0] for i in range(len(tr) - 1)]
    out = {"frames": k, "download": download, "shard": f"{k_sh}/{n_sh}", "wall_ms_per_frame": round(wall, 4),
           "trace_ms_median": round(statistics.median(e - s for s, e in tr), 4),
           "trace_period_ms_median": round(statistics.median(period), 4),
           "gap_ms": [round(g, 4) for g in gaps],
           "render_end_after_trace_end_ms": [round(rd[i][1] - tr[i][1], 4) for i in range(min(len(rd), len(tr)))],
           "render_start_before_trace_start_ms": [round(tr[i][0] - rd[i][0], 4) for i in range(min(len(rd), len(tr)))]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
