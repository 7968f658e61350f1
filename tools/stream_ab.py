"""A/B of bench.py's streamed frame loop under environment variants, no profiler attached
(rocprofv3's kernel trace changes how the frames overlap). Each variant runs in its own
process: K frames of shard S of N of the headline workload enqueued back to back, each
with its gather (mode), one wait at the end; variants interleaved `reps` times; median
ms per frame reported, every variant's frame hash checked against the first one's.

    python tools/stream_ab.py [--reps 3] [--frames 20] [--shards N] [--shard S] \
        "name:ENV=V,ENV2=V2:mode" ...        mode: gather (default) | u8 | none
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))

CHILD = r'''
import ctypes as C, hashlib, json, os, sys, time
sys.path.insert(0, os.path.join(sys.argv[1], "fo-rma_amd"))
import forma_rt as fr
mode, frames, n, k = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
sc = fr.Scene.from_file(fr.scene_path("scene_08"), 1920, 1080)
p = fr.make_params(1920, 1080, 256, 8, shard_index=k, shard_count=n, scene_jit="wait")
ctx = fr.RenderContext(0)
frame = fr.PinnedFrame(1920, 1080)
ctx.prepare(sc, sc.camera, p)
def run(m):
    for _ in range(m):
        ctx.render(sc, sc.camera, p)
        if mode == "gather":
            ctx.download_async(frame)
        elif mode == "u8":
            fr.check(fr.lib().fr_ctx_download_async(ctx._h, None, frame.u8.ctypes.data_as(C.POINTER(C.c_uint8))))
    ctx.wait()
run(3)
ctx.trace_log(True)
t = time.perf_counter()
run(frames)
ms = (time.perf_counter() - t) / frames * 1e3
tl = ctx.trace_log_read()
st = ctx.sync()
mean, _ = ctx.download(1920, 1080)
dev = {}
try:
    import torch
    dev["hbm_gb"] = round(torch.cuda.get_device_properties(0).total_memory / 2**30, 1)
except Exception:
    pass
print(json.dumps({"ms": ms, "trace_ms": sum(tl) / len(tl), "occupancy": st["occupancy"],
                  "sha": hashlib.sha256(mean.tobytes()).hexdigest()[:16], **dev}))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("variants", nargs="+")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--shards", type=int, default=1)
    ap.add_argument("--shard", type=int, default=0)
    ap.add_argument("--allow-diff", action="append", default=[],
                    help="variant whose frame may differ (a measurement-only build)")
    a = ap.parse_args()
    specs = []
    for v in a.variants:
        parts = v.split(":")
        name = parts[0]
        env = dict(kv.split("=", 1) for kv in parts[1].split(",") if kv) if len(parts) > 1 else {}
        mode = parts[2] if len(parts) > 2 and parts[2] else "gather"
        specs.append((name, env, mode))
    res = {s[0]: [] for s in specs}
    ref = None
    for rep in range(a.reps):
        for name, env, mode in specs:
            e = dict(os.environ, **env)
            out = subprocess.run([sys.executable, "-c", CHILD, ROOT, mode, str(a.frames), str(a.shards), str(a.shard)],
                                 env=e, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(json.dumps({"variant": name, "error": out.stderr[-600:]}), flush=True)
                sys.exit(1)
            r = json.loads(out.stdout.strip().splitlines()[-1])
            if name not in a.allow_diff:
                ref = ref or r["sha"]
            if r["sha"] != ref and name not in a.allow_diff:
                print(json.dumps({"variant": name, "error": f"frame hash {r['sha']} != {ref}"}), flush=True)
                sys.exit(1)
            res[name].append(r)
            print(json.dumps({"rep": rep, "variant": name, **r}), flush=True)
    for name, rs in res.items():
        ms = sorted(r["ms"] for r in rs)
        tr = sorted(r["trace_ms"] for r in rs)
        print(json.dumps({"variant": name, "median_ms_per_frame": round(ms[len(ms) // 2], 4),
                          "median_trace_ms": round(tr[len(tr) // 2], 4), "runs": len(rs)}), flush=True)


if __name__ == "__main__":
    main()
