"""FR_DIAG counters of shard 0 of N of the headline frame (FORMA_RT_LIB=an FR_DIAG build):
python tools/diag_shard.py [N] [ENV=VALUE ...]"""
import os
import sys
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "fo-rma_amd"))
for kv in sys.argv[2:]:
    k, _, v = kv.partition("=")
    os.environ[k] = v
import forma_rt as fr  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
sc = fr.Scene.from_file(fr.scene_path("scene_08"), 1920, 1080)
ctx = fr.RenderContext(0)
p = fr.make_params(1920, 1080, 256, 8, shard_index=0, shard_count=n)
for _ in range(2):
    ctx.render(sc, sc.camera, p)
    st = ctx.sync()
print(sys.argv[1:], st, flush=True)
