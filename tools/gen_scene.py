"""Scene generator: the reference generator's grid formula, parameterised.

Restates python-extras/scene_generator.py:54-86 — `count` objects on a 10-wide
grid 5 units apart, rotation (0.46193978, 0.1913417, 0.1913417, 0.84462326),
scale 5, camera (0, 2, -12) fov 60 — with the mesh and count as options, and
serialises it the way the reference does (json.dump(asdict(scene), indent=4)).
With --count 100 --mesh cube the bytes equal the reference generator's output
(tests/golden/generator_100_cubes.json). Config 5 uses --count 10000 --mesh sphere.

    python tools/gen_scene.py --count 10000 --mesh sphere --out /tmp/spheres.json
"""
import argparse
import json
import math


def generator_scene(count=100, mesh="cube", material="DiffuseColorMaterial", name="scene_08"):
    objects = [{
        "mesh": mesh,
        "material": material,
        "position": {"x": i % 10 * 5.0, "y": math.floor(i / 10) * 5.0, "z": 0.0},
        "rotation": {"x": 0.46193978, "y": 0.1913417, "z": 0.1913417, "w": 0.84462326},
        "scale": {"x": 5.0, "y": 5.0, "z": 5.0},
    } for i in range(count)]
    return {
        "name": name,
        "camera": {"position": {"x": 0.0, "y": 2.0, "z": -12.0},
                   "rotation": {"x": 0.0, "y": 0.0, "z": 0.0, "w": 1.0}, "fov": 60.0},
        "lights": [{"color": {"x": 0.0, "y": 0.0, "z": 0.0}, "intensity": 1.0,
                    "position": {"x": 0.0, "y": 0.0, "z": 0.0},
                    "rotation": {"x": 0.0, "y": 0.0, "z": 0.0, "w": 0.0},
                    "scale": {"x": 0.0, "y": 0.0, "z": 0.0}}],
        "objects": objects,
    }


def dumps(scene):
    return json.dumps(scene, indent=4)


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--count", type=int, default=100)
    ap.add_argument("--mesh", default="cube")
    ap.add_argument("--material", default="DiffuseColorMaterial")
    ap.add_argument("--out", default="-")
    a = ap.parse_args()
    text = dumps(generator_scene(a.count, a.mesh, a.material))
    if a.out == "-":
        print(text, end="")
    else:
        with open(a.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
