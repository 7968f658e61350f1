"""Bundle the reference's scene files as input data for the GPU box.

The GPU box only receives this repository, so the scenes the configs name
(scenes/scene_01.json, scene_08.json, ...) are carried as data under
fo-rma_amd/scenes/. Whitespace outside strings is stripped; every token —
in particular every number's source text — is kept byte for byte, so strtof
parses exactly what the reference's serde_json would.

Run in the build container only (reads /root/reference):
    python tools/vendor_scenes.py
"""
import glob
import os
import sys

SRC = "/root/reference/scenes"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "fo-rma_amd", "scenes")


def minify(text):
    out, in_str, esc = [], False, False
    for ch in text:
        if in_str:
            out.append(ch)
            if esc:
                esc = False
            elif ch == "\\":
                esc = True
            elif ch == '"':
                in_str = False
        elif ch == '"':
            in_str = True
            out.append(ch)
        elif ch not in " \t\r\n":
            out.append(ch)
    return "".join(out)


def main():
    if not os.path.isdir(SRC):
        sys.exit(f"{SRC} not present (this script runs in the build container only)")
    os.makedirs(DST, exist_ok=True)
    for path in sorted(glob.glob(os.path.join(SRC, "*.json"))):
        name = os.path.splitext(os.path.basename(path))[0]
        with open(path) as f:
            text = minify(f.read())
        with open(os.path.join(DST, f"{name}.min.json"), "w") as f:
            f.write(text + "\n")
        print(name, len(text))


if __name__ == "__main__":
    main()
