"""Scene-specialised kernel (FR_FLAG_SCENE_JIT) against the compiled-in one on the GPU:
same bits, and the compile / cache timings (tools for the GPU box, not a test)."""
import hashlib
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fo-rma_amd"))
import forma_rt as fr  # noqa: E402


def run(scene, w, h, spp, depth, jit):
    sc = fr.Scene.from_file(fr.scene_path(scene), w, h) if not scene.startswith("builtin") else fr.Scene.builtin(
        int(scene[-1]), w, h)
    ctx = fr.RenderContext(0)
    t0 = time.perf_counter()
    ctx.render(sc, sc.camera, fr.make_params(w, h, spp, depth, scene_jit=jit))
    st = ctx.sync()
    dt = time.perf_counter() - t0
    mean, u8 = ctx.download(w, h)
    info = ctx.jit_info()
    ctx.close()
    return hashlib.sha256(mean.tobytes()).hexdigest()[:16], st, info, dt


for scene in sys.argv[1:] or ["scene_08", "scene_01", "scene_03", "scene_07"]:
    a = run(scene, 320, 180, 32, 8, False)
    b = run(scene, 320, 180, 32, 8, True)
    c = run(scene, 320, 180, 32, 8, True)
    same = a[0] == b[0] == c[0] and a[1]["segments"] == b[1]["segments"]
    print(f"{scene}: {'SAME' if same else 'DIFFERENT'} aot {a[0]} jit {b[0]} info1 {b[2]} first {b[3]*1e3:.0f} ms, "
          f"info2 {c[2]} second {c[3]*1e3:.0f} ms", flush=True)
