"""Run an FR_DIAG build (FORMA_RT_LIB=...) and print its phase counters.

    python tools/diag_run.py [scene W H SPP] ...   (default: two small cases)"""
import os
import sys
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "fo-rma_amd"))
import forma_rt as fr

cases = [("scene_08", 480, 270, 64), ("scene_01", 480, 270, 16)]
if len(sys.argv) > 1:
    a = sys.argv[1:]
    cases = [(a[i], int(a[i + 1]), int(a[i + 2]), int(a[i + 3])) for i in range(0, len(a), 4)]
for scene, w, h, spp in cases:
    if scene.startswith("gen:"):  # gen:COUNT:MESH, the generator scene (tools/gen_scene.py)
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import gen_scene
        _, count, mesh = scene.split(":")
        sc = fr.Scene.from_json(gen_scene.dumps(gen_scene.generator_scene(int(count), mesh)), w, h)
    else:
        sc = fr.Scene.from_file(fr.scene_path(scene), w, h)
    m, u, st = fr.render(sc, sc.camera, w, h, spp, 8)
    print(scene, w, h, spp, st, flush=True)
