"""Pin tools/gen_scene.py against the reference's own scene generator.

Imports python-extras/scene_generator.py from the read-only reference checkout
(build container only), builds the 100-cube scene exactly as its __main__ block
does (python-extras/scene_generator.py:54-86), serialises it with the module's
own save_scene_to_file into a temporary file, and records the output's size and
sha256 in generator_100_cubes.json. The reference module itself is not copied.
"""
import hashlib
import importlib.util
import json
import math
import os
import tempfile

REF = "/root/reference/python-extras/scene_generator.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "generator_100_cubes.json")


def main():
    spec = importlib.util.spec_from_file_location("ref_scene_generator", REF)
    g = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(g)  # __main__ guard: import has no side effects
    camera = g.Camera(position=g.Vec3(0.0, 2.0, -12.0), rotation=g.Quaternion(0.0, 0.0, 0.0, 1.0), fov=60.0)
    light = g.Light(color=g.Vec3(0.0, 0.0, 0.0), intensity=1.0, position=g.Vec3(0.0, 0.0, 0.0),
                    rotation=g.Quaternion(0.0, 0.0, 0.0, 0.0), scale=g.Vec3(0.0, 0.0, 0.0))
    objects = [g.SceneObject(mesh="cube", material="DiffuseColorMaterial",
                             position=g.Vec3(i % 10 * 5.0, math.floor(i / 10) * 5.0, 0.0),
                             rotation=g.Quaternion(0.46193978, 0.1913417, 0.1913417, 0.84462326),
                             scale=g.Vec3(5.0, 5.0, 5.0)) for i in range(100)]
    scene = g.Scene(name="scene_08", camera=camera, lights=[light], objects=objects)
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "scene.json")
        g.save_scene_to_file(scene, path)
        data = open(path, "rb").read()
    rec = {"generator": "python-extras/scene_generator.py:54-86 (count=100, mesh=cube)",
           "bytes": len(data), "sha256": hashlib.sha256(data).hexdigest()}
    with open(OUT, "w") as f:
        json.dump(rec, f, indent=2)
    print(rec)


if __name__ == "__main__":
    main()
