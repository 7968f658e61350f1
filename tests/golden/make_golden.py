"""Golden image fixtures from the oracle (oracle/oracle.cpp), for the parity tests.

Each case renders a small image with save_image semantics (tracer.rs:160-187)
and stores the f32 means, the u8 image and the path counters. The oracle is
pinned first by tests/test_oracle_kat.py (the reference's Vec3 KATs and analytic
cases); these fixtures then freeze its output so that oracle regressions and
GPU-vs-fixture drift are both caught. Re-generate only after a deliberate
semantic change:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, ROOT)
from oracle import oracle_py, scene_ref  # noqa: E402

SCENES = os.path.join(ROOT, "fo-rma_amd", "scenes")
OUT = os.path.dirname(os.path.abspath(__file__))

# name: (scene, width, height, spp, max_depth, seed)
CASES = {
    "scene07_empty_32x32_s2_d4": ("json:scene_07", 32, 32, 2, 4, 0x5EED),
    "simple_32x24_s4_d8": ("builtin:0", 32, 24, 4, 8, 0x5EED),
    "objects_32x32_s4_d8": ("builtin:2", 32, 32, 4, 8, 0x5EED),
    "frontend_32x32_s4_d50": ("builtin:3", 32, 32, 4, 50, 0x5EED),
    "scene01_64x64_s2_d4": ("json:scene_01", 64, 64, 2, 4, 0x5EED),
    "scene03_obb_32x32_s4_d4": ("json:scene_03", 32, 32, 4, 4, 0x5EED),
    "scene08_64x36_s4_d8": ("json:scene_08", 64, 36, 4, 8, 0x5EED),
    "scene08_33x17_s3_d8_seed7": ("json:scene_08", 33, 17, 3, 8, 7),
    "scene02_mesh_48x27_s3_d8": ("json:scene_02", 48, 27, 3, 8, 0x5EED),
    "scene06_cyl_48x27_s2_d8": ("json:scene_06", 48, 27, 2, 8, 0x5EED),
    "scene09_tet_40x40_s4_d8": ("json:scene_09", 40, 40, 4, 8, 0x5EED),
    # 37 spp: two 16-sample streams, then the last block as sub-block streams of 4, 1
    "scene08_24x16_s37_d8": ("json:scene_08", 24, 16, 37, 8, 0x5EED),
}


def scene_and_camera(spec, w, h):
    kind, name = spec.split(":")
    if kind == "builtin":
        return scene_ref.BUILTIN[int(name)](), oracle_py.camera_new(w, h)
    with open(os.path.join(SCENES, f"{name}.min.json")) as f:
        prims, (frm, at, vup, fov) = scene_ref.load_json(f.read())
    return prims, oracle_py.camera_look(frm, at, vup, fov, 0.1, w, h)


def render_case(name):
    spec, w, h, spp, depth, seed = CASES[name]
    prims, cam = scene_and_camera(spec, w, h)
    mean, u8, cnt, _ = oracle_py.render(prims, cam, w, h, spp, depth, seed=seed, threads=8)
    return mean, u8, cnt


def main():
    import sys
    names = sys.argv[1:] or list(CASES)  # regenerate only the named cases if given
    for name in names:
        mean, u8, cnt = render_case(name)
        np.savez_compressed(os.path.join(OUT, f"{name}.npz"), mean=mean, u8=u8,
                            counters=np.array([cnt["segments"], cnt["hits"], cnt["samples"], cnt["scatters"]],
                                              dtype=np.uint64))
        print(name, cnt)


if __name__ == "__main__":
    main()
