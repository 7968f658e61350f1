import os, sys
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "fo-rma_amd"))
import forma_rt as fr
for scene, w, h, spp in [("scene_08", 480, 270, 64), ("scene_01", 480, 270, 16)]:
    sc = fr.Scene.from_file(fr.scene_path(scene), w, h)
    m, u, st = fr.render(sc, sc.camera, w, h, spp, 8)
    print(scene, st, flush=True)
