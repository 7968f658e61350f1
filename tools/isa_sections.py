"""Per-phase VALU breakdown of the headline trace kernel (the scene_08 scene-specialised build).

Static side: trace_kernel.h is compiled the way jit.cpp's hiprtc build compiles it (same
options, the host build's tuning macros, scene_08's records as constants), with
-DFR_SEC_MARKS, which turns every SEC(k) region marker of the lane loop into an assembler
comment. The ISA listing is cut at those comments and each region's VALU instructions
are counted (v_* opcodes; SALU, LDS and memory instructions separately).

Dynamic side: an FR_SECCNT build of the library counts how many times a wave enters each
region per launch (the FR_SECCNT line on stderr, captured on the GPU box).

    python tools/isa_sections.py isa [--template=1,0,9,8,0,0,2,1] [--nojit] [--scene=scene_08] [--prelude=FILE] [-DNAME=V]  -> static table (JSON)
      (--nojit: the compiled-in kernel, e.g. --template=2,0,4,8,1,0,0,1 --nojit for C5's BVH kernel)
    python tools/isa_sections.py combine STATIC.json SECCNT_LINE_FILE SEGMENTS VALU_MEASURED [GRABS]

combine multiplies the two: VALU instructions per region per launch, their share, and the
lane-slots per segment (x 64 / segments). ISA_NOMARKS=1 compiles without the markers (the
product kernel's exact registers: the markers' asm statements can change allocation)."""
import json
import os
import re
import struct
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "fo-rma_amd", "csrc")
# counted regions, in trace_kernel.h's SC_* order
# (the BVH walk's scalar and vector paths are separate regions: SC_NODES / SC_NODEV after the
# node step's common head SC_NODE, SC_LTESTS / SC_LTESTV for one leaf test)
REGIONS = ["SC_ITER", "SC_CLAIM", "SC_JIT", "SC_NEED", "SC_REJ", "SC_CAM", "SC_SCAT", "SC_HIT", "SC_SKY", "SC_SHADE",
           "SC_END", "SC_NODE", "SC_LEAF", "SC_NODES", "SC_NODEV", "SC_LTESTS", "SC_LTESTV", "SC_LIST", "SC_LROOT"]
# marker-only regions: the counted region whose entries they share
DERIVED = {"SC_SETUP": "SC_CLAIM", "SC_ACC": "SC_NEED", "SC_POSTHIT": "SC_HIT", "SC_POSTSHADE": "SC_ITER",
           "SC_LATCH": "SC_ITER", "SC_NODET": "SC_NODE"}
# render.hip jit_defines() for the default build
DEFINES = dict(FR_KREJ=4, FR_KREJ_NIB=9, FR_CLAIM_MIN=1, FR_CLAIM_MIN_NIB=3, FR_NUM_SGPR=96, FR_BLOCK_SAMPLES=16,
               FR_FINE_SAMPLES=4, FR_STAGE=4, FR_BVH_STAGE=2, FR_NIB_WAVES=8, FR_DIFF12_WAVES=7)
OPTS = ["-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fhip-fp32-correctly-rounded-divide-sqrt",
        "-fno-gpu-flush-denormals-to-zero", "-fno-slp-vectorize"]


def scene_records(name="scene_08"):
    """The scene's 64-B device records as render.hip upload_scene lays them out (spheres,
    boxes and planes; the kind in g3.w)."""
    sys.path.insert(0, os.path.join(ROOT, "fo-rma_amd"))
    import forma_rt as fr
    sc = fr.Scene.from_file(fr.scene_path(name), 64, 36)
    words = []
    for p in sc.prims():
        g = list(p.g)
        if p.kind == fr.FR_SPHERE:
            f = g[0:4] + [0.0] * 12
        elif p.kind == fr.FR_AABB:
            f = g[0:3] + [0.0] + g[3:6] + [0.0] * 9
        elif p.kind == fr.FR_PLANE:
            f = g[0:3] + [0.0] + g[3:6] + [0.0] + g[6:9] + [0.0] * 5
        else:
            raise SystemExit(f"isa_sections: kind {p.kind} not laid out here")
        rec = list(struct.unpack("16I", struct.pack("16f", *f)))
        rec[15] = p.kind
        words.append(rec)
    return words


def build_isa(targs, extra_defs=(), jit=True, scene="scene_08", prelude_file=None):
    out = os.path.join(ROOT, "fo-rma_amd", "build", "isa_jit")
    os.makedirs(out, exist_ok=True)
    defs = dict(DEFINES)
    for a in extra_defs:  # -DNAME=V overrides the host build's value of NAME
        if a.startswith("-D") and "=" in a and a[2:].split("=", 1)[0] in defs:
            defs[a[2:].split("=", 1)[0]] = a.split("=", 1)[1]
    pre = "".join(f"#define {k} {v}\n" for k, v in defs.items())
    if jit:  # the scene-specialised build (scene_08's records); else the compiled-in kernel
        recs = scene_records(scene)
        pre += f"#define FR_JIT_N {len(recs)}u\n#define FR_JIT_REC " + ",".join(
            "{" + ",".join(f"0x{w:08x}u" for w in r) + "}" for r in recs) + "\n"
    if prelude_file:  # e.g. the FR_JIT_CLU_* cluster constants render.hip adds for a scene
        pre += open(prelude_file).read()
    ta = targs
    inst = (f"template __global__ void fr::trace_kernel<{ta[0]}, {'true' if ta[1] else 'false'}, {ta[2]}, {ta[3]}, "
            f"{'true' if ta[4] else 'false'}, {'true' if ta[5] else 'false'}, {ta[6]}, {ta[7]}>(fr::KArgs);\n")
    src = os.path.join(out, (scene.replace("_", "") + "_kernel.hip") if jit else "kernel_%s.hip" % "_".join(map(str, targs)))
    with open(src, "w") as f:
        f.write(pre + '#include "trace_kernel.h"\n' + inst)
    asm = src[:-4] + ".s"
    extra_defs = [a for a in extra_defs if not (a.startswith("-D") and "=" in a and a[2:].split("=", 1)[0] in defs)]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "--cuda-device-only", "-S", "-I", CSRC, "-I",
           os.path.join(ROOT, "include"), *OPTS, *([] if os.environ.get("ISA_NOMARKS") else ["-DFR_SEC_MARKS"]),
           *extra_defs, src, "-o", asm]
    subprocess.run(cmd, check=True)
    return asm


def count_regions(asm):
    """VALU / SALU / LDS / memory instructions per region. A marker labels its basic block
    (the assembler comment may sit anywhere in the block); an unmarked block takes the
    region of the block before it in the layout, except: blocks of the rejection loop
    (the loops nested in the lane loop) are SC_REJ / SC_LENS; lane-loop blocks laid out before the
    loop header are SC_LATCH; unmarked blocks with a full IEEE division (v_div_fixup: the
    reciprocal guard's and the sky parameter's fallbacks) are RARE (not entered in a normal
    frame); blocks after the lane loop are EPILOGUE. `instances` counts a region's marker
    copies (unrolled loops)."""
    lines = open(asm).read().splitlines()
    blocks, cur, in_fn, meta = [], None, False, {}
    for ln in lines:
        s = ln.strip()
        for key in ("vgpr_count", "sgpr_count", "sgpr_spill_count", "vgpr_spill_count"):
            m = re.search(r"\." + key + r":\s+(\d+)", s)
            if m:
                meta[key] = int(m.group(1))
        if re.match(r"^_ZN2fr12trace_kernel\S*:", s):
            in_fn = True
            cur = {"name": "entry", "mark": None, "cmt": "", "ops": []}
            blocks.append(cur)
            continue
        if not in_fn:
            continue
        if s.startswith(".Lfunc_end"):
            in_fn = False
            continue
        m = re.match(r"^(\.LBB\d+_\d+):|^; (%bb\.\d+):", s)
        if m:
            cur = {"name": m.group(1) or m.group(2), "mark": None, "cmt": s, "ops": []}
            blocks.append(cur)
            continue
        if s.startswith(";") and "Loop" in s:
            cur["cmt"] += " " + s
        m = re.search(r";FRSEC (\w+)", s)
        if m:
            cur["mark"] = m.group(1)
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        cur["ops"].append(s.split()[0])
    # the lane loop's header is the block marked SC_ITER; the rejection loop's blocks name
    # the inner loop's header in their comments
    hdr = next(b["name"] for b in blocks if b["mark"] == "SC_ITER")
    lane_loop = "Header=" + hdr.lstrip(".").replace("LBB0_", "BB0_")
    inner = {}  # inner loop header -> its region (the blocks of each loop name their header)
    for b in blocks:
        if b["mark"] in ("SC_REJ", "SC_LENS"):
            inner[b["name"].lstrip(".").replace("LBB0_", "BB0_")] = b["mark"]
    region, seen_hdr, done = "PROLOGUE", False, False
    tab = {}
    for b in blocks:
        in_lane = lane_loop in b["cmt"] or ("Parent Loop " + hdr.lstrip(".").replace("LBB0_", "BB0_")) in b["cmt"] or (
            seen_hdr and "Depth=" in b["cmt"])
        if b["name"] == hdr:
            seen_hdr = True
        if b["mark"]:
            region = b["mark"]
        elif seen_hdr and not in_lane and b["name"] != hdr:
            region, done = "EPILOGUE", True
        elif in_lane and not seen_hdr:
            region = "SC_LATCH"
        r = region
        for h, reg in inner.items():
            if ("Header=" + h + " ") in (b["cmt"] + " ") and not b["mark"]:
                r = reg
        # (the sky parameter's IEEE fallback too: its fast path is the default since round 5)
        if not b["mark"] and "v_div_fixup_f32" in b["ops"]:
            r = "RARE"
        t = tab.setdefault(r, {"valu": 0, "salu": 0, "lds": 0, "mem": 0, "blocks": 0, "instances": 0})
        t["blocks"] += 1
        if b["mark"]:
            t["instances"] += 1  # copies of the marker (an unrolled loop repeats its region)
        for op in b["ops"]:
            kind = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") else
                    "lds" if op.startswith("ds_") else "mem")
            t[kind] += 1
    return tab, meta


def combine(static_path, seccnt_path, segments, valu_measured, grabs=0):
    st = json.load(open(static_path))
    line = [ln for ln in open(seccnt_path) if "FR_SECCNT" in ln][-1]
    counts = json.loads(line.split("FR_SECCNT", 1)[1])
    lanes_l = [ln for ln in open(seccnt_path) if "FR_SECLANES" in ln]
    lanes = json.loads(lanes_l[-1].split("FR_SECLANES", 1)[1]) if lanes_l else [0] * len(counts)
    # a build with fewer regions (older SC_* lists) reads 0 for the later ones
    counts += [0] * (len(REGIONS) - len(counts))
    lanes += [0] * (len(REGIONS) - len(lanes))
    tab = st["regions"]
    rows, tot = [], 0.0
    for name in REGIONS + list(DERIVED) + ["SC_GRAB"]:
        # VALU per entry: a region's instructions over its marker's copies (each copy of an
        # unrolled loop body counts its own entries)
        v = tab.get(name, {}).get("valu", 0) / max(1, tab.get(name, {}).get("instances", 1))
        if name in REGIONS:
            n, ln = counts[REGIONS.index(name)], lanes[REGIONS.index(name)]
        elif name in DERIVED:
            n, ln = counts[REGIONS.index(DERIVED[name])], lanes[REGIONS.index(DERIVED[name])]
        else:
            n, ln = grabs, 0
        rows.append((name, v, n, v * n, ln))
        tot += v * n
    out = {"regions": [], "total_valu_model": tot, "valu_measured": valu_measured,
           "model_over_measured": tot / valu_measured if valu_measured else None, "segments": segments}
    for name, v, n, vn, ln in rows:
        # active lanes per entry, and the region's idle lane-slots: VALU x (64 - active lanes)
        act = ln / n if n and ln else None
        out["regions"].append({"region": name, "static_valu": v, "wave_entries": n, "valu": vn,
                               "share": vn / tot if tot else 0.0, "lane_slots_per_segment": vn * 64.0 / segments,
                               "active_lanes_per_entry": round(act, 2) if act else None,
                               "idle_lane_slots": v * (64.0 * n - ln) if ln else None})
    return out


if __name__ == "__main__":
    if sys.argv[1] == "isa":
        targs = [1, 0, 9, 8, 0, 0, 2, 1]
        extra = []
        jit = True
        scene = "scene_08"
        prelude_file = None
        for a in sys.argv[2:]:
            if a.startswith("--template="):
                targs = [int(x) for x in a.split("=", 1)[1].split(",")]
            elif a == "--nojit":
                jit = False
            elif a.startswith("--scene="):
                scene = a.split("=", 1)[1]
            elif a.startswith("--prelude="):
                prelude_file = a.split("=", 1)[1]
            elif a.startswith("-D"):
                extra.append(a)
        asm = build_isa(targs, extra, jit, scene, prelude_file)
        tab, meta = count_regions(asm)
        print(json.dumps({"template": targs, "asm": os.path.relpath(asm, ROOT), "meta": meta, "regions": tab},
                         indent=1))
    elif sys.argv[1] == "combine":
        g = float(sys.argv[6]) if len(sys.argv) > 6 else 0.0
        print(json.dumps(combine(sys.argv[2], sys.argv[3], float(sys.argv[4]), float(sys.argv[5]), g), indent=1))
