"""Time one render of a configuration on GPU 0:
python tools/time_config.py SCENE W H SPP DEPTH [reps [shards]]   (shards: time shard 0 of that many)
SCENE is a bundled scene name or gen:<count>:<mesh> (tools/gen_scene.py)."""
import json
import os
import sys
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fo-rma_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import forma_rt as fr

name, w, h, spp, depth = sys.argv[1], *map(int, sys.argv[2:6])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 3
shards = int(sys.argv[7]) if len(sys.argv) > 7 else 1
if name.startswith("gen:"):
    import gen_scene
    _, count, mesh = name.split(":")
    sc = fr.Scene.from_json(gen_scene.dumps(gen_scene.generator_scene(int(count), mesh)), w, h)
else:
    sc = fr.Scene.from_file(fr.scene_path(name), w, h)
ctx = fr.RenderContext(0)
p = fr.make_params(w, h, spp, depth, shard_index=0, shard_count=shards)
ms = []
for _ in range(reps):
    ctx.render(sc, sc.camera, p)
    st = ctx.sync()
    ms.append(st["kernel_ms"])
st["kernel_ms_median"] = sorted(ms)[len(ms) // 2]
st["msamples_per_s"] = st["samples"] / st["kernel_ms_median"] / 1e3
print(json.dumps({"scene": name, "w": w, "h": h, "spp": spp, "depth": depth, "shard": f"0/{shards}", "prims": len(sc),
                  **st}), flush=True)
