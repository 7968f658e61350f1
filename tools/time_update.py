"""Frame time of the interactive path, tracer.rs:30-55 update(): one 1-spp frame of the
simple scene (get_simple_scene, max_depth 50) with an orbiting camera, on the model's
persistent render context, including the u8 download into model.pixels.

    python tools/time_update.py [W H] [frames]

Prints one JSON line: median / p90 host wall time per update() call, and the same frame
through the one-shot fr_render_hip (a context made and freed per call) for comparison."""
import json
import os
import sys
import time

ROOT = os.environ.get("GRAFT_REPO_ROOT", os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fo-rma_amd"))
import forma_rt as fr  # noqa: E402


def main():
    w, h = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (1920, 1080)
    frames = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    m = fr.create_model(w, h)
    fr.update(m, 0b001000, 1.0 / 60)  # first frame: context, scene upload, buffers
    ts = []
    for k in range(frames):
        t = time.perf_counter()
        fr.update(m, 0b001000 if k % 2 else 0b000100, 1.0 / 60)
        ts.append((time.perf_counter() - t) * 1e3)
    st = m.last_stats
    one = []
    for _ in range(5):
        t = time.perf_counter()
        fr.render(m.scene, m.scene.camera, w, h, 1, fr.MAX_DEPTH, 1234)
        one.append((time.perf_counter() - t) * 1e3)
    ts.sort()
    one.sort()
    print(json.dumps({"workload": f"update() simple scene {w}x{h} 1spp depth 50", "frames": frames,
                      "ms_median": round(ts[len(ts) // 2], 3), "ms_p90": round(ts[int(0.9 * len(ts))], 3),
                      "kernel_ms": round(st["kernel_ms"], 3), "fps_median": round(1e3 / ts[len(ts) // 2], 1),
                      "one_shot_render_ms_median": round(one[len(one) // 2], 3),
                      "segments_per_sample": round(st["segments"] / st["samples"], 3)}), flush=True)
    m.close()


if __name__ == "__main__":
    main()
