"""Render the headline frame (C3: scene_08 1920x1080, 256 spp, depth 8, scene kernel) once
with an FR_SECCNT build (FORMA_RT_LIB=...): stderr gets the FR_SECCNT line (wave entries per
lane-loop region, tools/isa_sections.py), stdout the frame's counters as JSON.

    FORMA_RT_LIB=fo-rma_amd/build/ab/libforma_rt_seccnt.so python tools/seccnt_run.py [W H SPP]"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "fo-rma_amd"))
import forma_rt as fr  # noqa: E402

w, h, spp = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (1920, 1080, 256)))
sc = fr.Scene.from_file(fr.scene_path("scene_08"), w, h)
m, u, st = fr.render(sc, sc.camera, w, h, spp, 8, scene_jit="wait")
print(json.dumps({"w": w, "h": h, "spp": spp, **st}), flush=True)
