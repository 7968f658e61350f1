"""Render the headline frame (C3: scene_08 1920x1080, 256 spp, depth 8, scene kernel) once
with an FR_SECCNT build (FORMA_RT_LIB=...): stderr gets the FR_SECCNT line (wave entries per
lane-loop region, tools/isa_sections.py), stdout the frame's counters as JSON.

    FORMA_RT_LIB=fo-rma_amd/build/ab/libforma_rt_seccnt.so python tools/seccnt_run.py [SCENE] [W H SPP]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fo-rma_amd"))
import forma_rt as fr  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].isdigit() else "scene_08"
nums = [int(x) for x in sys.argv[1:] if x.isdigit()]
w, h, spp = nums[:3] if len(nums) >= 3 else (1920, 1080, 256)
if name.startswith("gen:"):  # gen:COUNT:MESH, the generator scene (BASELINE config C5: gen:10000:sphere 1920 1080 512)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import gen_scene
    _, count, mesh = name.split(":")
    sc = fr.Scene.from_json(gen_scene.dumps(gen_scene.generator_scene(int(count), mesh)), w, h)
else:
    sc = fr.Scene.from_file(fr.scene_path(name), w, h)
m, u, st = fr.render(sc, sc.camera, w, h, spp, 8, scene_jit="wait")
print(json.dumps({"w": w, "h": h, "spp": spp, **st}), flush=True)
