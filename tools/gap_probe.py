"""Gaps between streamed frames' trace kernels: K frames of the headline workload on one
context, enqueued back to back (bench.py's loop), with or without each frame's gather.
Run under `rocprofv3 --kernel-trace` and read the CSV with --analyze, which prints, per
frame, the trace kernel's duration and the idle time before the next trace starts, and
what ran in that gap.

    python tools/gap_probe.py MODE [K]       MODE: gather | u8 | none
    python tools/gap_probe.py --analyze KERNEL_TRACE.csv
"""
import csv
import json
import os
import sys
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fo-rma_amd"))


def analyze(path):
    rows = list(csv.DictReader(open(path)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r["Queue_Id"]) for r in rows)
    traces = [k for k in ks if "trace_kernel" in k[2]]
    gaps = []
    for a, b in zip(traces, traces[1:]):
        between = [(round((s - a[1]) / 1e3, 1), round((e - s) / 1e3, 1), n.split("(")[0][-28:], q)
                   for s, e, n, q in ks if a[1] <= s < b[0] or (s < b[0] and e > a[1] and "trace" not in n)]
        gaps.append({"trace_ms": round((a[1] - a[0]) / 1e6, 4), "gap_us": round((b[0] - a[1]) / 1e3, 1),
                     "between": between[:8]})
    for g in gaps:
        print(json.dumps(g))
    steady = gaps[len(gaps) // 2:]
    print(json.dumps({"frames": len(traces), "mean_trace_ms": round(sum(g["trace_ms"] for g in steady) / len(steady), 4),
                      "mean_gap_us": round(sum(g["gap_us"] for g in steady) / len(steady), 1)}))


def main():
    if sys.argv[1] == "--analyze":
        return analyze(sys.argv[2])
    import forma_rt as fr
    mode = sys.argv[1]
    k = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    sc = fr.Scene.from_file(fr.scene_path("scene_08"), 1920, 1080)
    p = fr.make_params(1920, 1080, 256, 8, scene_jit="wait")
    ctx = fr.RenderContext(0)
    frame = fr.PinnedFrame(1920, 1080)
    ctx.prepare(sc, sc.camera, p)
    t = time.perf_counter()
    for _ in range(k):
        ctx.render(sc, sc.camera, p)
        if mode == "gather":
            ctx.download_async(frame)
        elif mode == "u8":  # the u8 image only (6 MB instead of 31 MB)
            import ctypes as C
            fr.check(fr.lib().fr_ctx_download_async(ctx._h, None, frame.u8.ctypes.data_as(C.POINTER(C.c_uint8))))
    ctx.wait()
    print(json.dumps({"mode": mode, "frames": k, "ms_per_frame": round((time.perf_counter() - t) / k * 1e3, 4)}))


if __name__ == "__main__":
    main()
