"""Render one configuration a few times on device 0: the program bench.py (and
tools/profile.sh) runs under `rocprofv3 --pmc` to read hardware counters of the trace
kernel. Prints one JSON line with the last frame's stats.

    python3 tools/pmc_frame.py SCENE W H SPP DEPTH [frames]

SCENE is a bundled scene name or gen:COUNT:MESH (tools/gen_scene.py, e.g. gen:10000:sphere
for BASELINE config C5).
"""
import json
import os
import sys

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fo-rma_amd"))
os.environ.setdefault("FR_NO_TORCH", "1")  # the profiled child needs no torch
import forma_rt as fr  # noqa: E402


def main():
    name, w, h, spp, depth = sys.argv[1], *map(int, sys.argv[2:6])
    frames = int(sys.argv[6]) if len(sys.argv) > 6 else 2
    if name.startswith("gen:"):
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import gen_scene
        _, count, mesh = name.split(":")
        sc = fr.Scene.from_json(gen_scene.dumps(gen_scene.generator_scene(int(count), mesh)), w, h)
    else:
        sc = fr.Scene.from_file(fr.scene_path(name), w, h)
    ctx = fr.RenderContext(0)
    p = fr.make_params(w, h, spp, depth)
    st = None
    for _ in range(frames):
        ctx.render(sc, sc.camera, p)
        st = ctx.sync()
    print(json.dumps({"scene": name, "w": w, "h": h, "spp": spp, "depth": depth, "frames": frames, **st}), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
