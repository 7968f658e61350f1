"""A/B timing of kernel variants (FORMA_RT_LIB builds of the same ABI) on one GPU.

    python tools/ab_bench.py lib1.so lib2.so ... [--reps 3] [--scene scene_08]

Each variant renders the bench workload; variants are interleaved `reps` times and the
median kernel time (HIP events) is reported. Every variant's image is checked bit-exact
against the first one's."""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))

CHILD = r'''
import json, os, sys, hashlib
sys.path.insert(0, os.path.join(sys.argv[1], "fo-rma_amd"))
import forma_rt as fr
scene, w, h, spp, depth, steps, shards = sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6]), int(sys.argv[7]), int(sys.argv[8])
if scene.startswith("gen:"):
    sys.path.insert(0, os.path.join(sys.argv[1], "tools"))
    import gen_scene
    _, count, mesh = scene.split(":")
    sc = fr.Scene.from_json(gen_scene.dumps(gen_scene.generator_scene(int(count), mesh)), w, h)
else:
    sc = fr.Scene.from_file(fr.scene_path(scene), w, h)
ctx = fr.RenderContext(0)
p = fr.make_params(w, h, spp, depth, shard_index=0, shard_count=shards)
ctx.render(sc, sc.camera, p); ctx.sync()
ms, tr = [], []
for _ in range(steps):
    ctx.render(sc, sc.camera, p); st = ctx.sync(); ms.append(st["kernel_ms"]); tr.append(st["trace_ms"])
mean, u8 = ctx.download(w, h)
print(json.dumps({"ms": sorted(ms)[len(ms)//2], "trace_ms": sorted(tr)[len(tr)//2],
                  "sha": hashlib.sha256(mean.tobytes()).hexdigest()[:16]}))
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--scene", default="scene_08")
    ap.add_argument("--size", default="1920x1080")
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--depth", type=int, default=8)
    ap.add_argument("--shards", type=int, default=1, help="time shard 0 of this many (one rank of N GPUs)")
    a = ap.parse_args()
    w, h = map(int, a.size.split("x"))
    res = {lib: [] for lib in a.libs}
    trace = {lib: [] for lib in a.libs}
    shas = {}
    for _ in range(a.reps):
        for lib in a.libs:
            # "lib.so@NAME=VALUE,..." runs that library with extra environment settings
            path, _, extra = lib.partition("@")
            env = dict(os.environ, FORMA_RT_LIB=os.path.abspath(path))
            for kv in filter(None, extra.split(",")):
                k, _, v = kv.partition("=")
                env[k] = v
            out = subprocess.run([sys.executable, "-c", CHILD, ROOT, a.scene, str(w), str(h), str(a.spp),
                                  str(a.depth), str(a.steps), str(a.shards)], env=env, capture_output=True, text=True, timeout=300)
            if out.returncode != 0:
                print(lib, "FAILED", out.stderr[-2000:])
                sys.exit(1)
            r = json.loads(out.stdout.strip().splitlines()[-1])
            res[lib].append(r["ms"])
            trace[lib].append(r.get("trace_ms", 0.0))
            shas[lib] = r["sha"]
    base = shas[a.libs[0]]
    for lib in a.libs:
        ms = sorted(res[lib])[len(res[lib]) // 2]
        tms = sorted(trace[lib])[len(trace[lib]) // 2]
        samples = w * h * a.spp / a.shards
        print(f"{os.path.basename(lib):40s} {ms:9.3f} ms (trace {tms:8.3f})  {samples / ms / 1e3:10.1f} Msamples/s  "
              f"{'same image' if shas[lib] == base else 'IMAGE DIFFERS ' + shas[lib]}")


if __name__ == "__main__":
    main()
