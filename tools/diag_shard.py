"""FR_DIAG run of one row shard of the bench workload: FORMA_RT_LIB=<diag build>
python tools/diag_shard.py SHARD SHARDS   (per-wave stamps go to $FR_DIAG_TIMES)"""
import os
import sys
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "fo-rma_amd"))
import forma_rt as fr

shard, shards = int(sys.argv[1]), int(sys.argv[2])
sc = fr.Scene.from_file(fr.scene_path("scene_08"), 1920, 1080)
ctx = fr.RenderContext(0)
p = fr.make_params(1920, 1080, 256, 8, shard_index=shard, shard_count=shards)
for _ in range(2):
    ctx.render(sc, sc.camera, p)
    st = ctx.sync()
print(shard, shards, st, flush=True)
