"""A one-shot caller's cost of the scene kernel, on a cold cache (tests/test_scene_jit.py
runs it in a fresh process with FR_JIT_CACHE pointing at an empty directory).

INTEGRATION.md's save_image through fr_mctx at 1920x1080, 50 samples (the reference's only
caller: frontend/macroquad.rs:60, save_image(&mut model, 50)), timed three ways on one
context set: the compiled-in kernel (flag off), the first FR_FLAG_SCENE_JIT render (no code
object anywhere: the compile is queued on the background thread and the render runs the
compiled-in kernel), and a render after the compile finished (the scene kernel). Every
image must be the same bits. Prints one JSON line.

    python tools/jit_cold.py [W H SPP] [--devices 0,0]
"""
import json
import os
import sys
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fo-rma_amd"))
import forma_rt as fr  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    w, h, spp = (int(args[0]), int(args[1]), int(args[2])) if len(args) >= 3 else (1920, 1080, 50)
    devices = [0]
    if "--devices" in sys.argv:
        devices = [int(d) for d in sys.argv[sys.argv.index("--devices") + 1].split(",")]
    sc = fr.Scene.from_file(fr.scene_path("scene_08"), w, h)
    mc = fr.MultiContext(devices)

    def frame(jit):
        t = time.perf_counter()
        mc.render(sc, sc.camera, fr.make_params(w, h, spp, 50, scene_jit=jit))
        mc.sync()
        ms = (time.perf_counter() - t) * 1e3
        return ms, mc.frame(), [mc.context(i).jit_state() for i in range(len(devices))]

    frame(False)  # buffers, scene upload, streams: the same for every variant below
    base_ms, (ref, ref_u8), _ = frame(False)
    cold_ms, (m1, u1), st1 = frame(True)
    t = time.perf_counter()
    fr.jit_wait()
    wait_ms = (time.perf_counter() - t) * 1e3
    hot_ms, (m2, u2), st2 = frame(True)
    same = all(bool((a.view("u4") == ref.view("u4")).all()) and bool((b == ref_u8).all())
               for a, b in ((m1, u1), (m2, u2)))
    print(json.dumps({"w": w, "h": h, "spp": spp, "devices": devices, "compiled_in_ms": round(base_ms, 3),
                      "cold_scene_jit_ms": round(cold_ms, 3), "cold_states": st1,
                      "ratio": round(cold_ms / base_ms, 3), "background_compile_left_ms": round(wait_ms, 1),
                      "scene_kernel_ms": round(hot_ms, 3), "hot_states": st2, "bit_identical": same}), flush=True)
    mc.close()


if __name__ == "__main__":
    main()
