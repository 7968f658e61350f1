"""VGPR liveness over a kernel's ISA listing (hipcc -S output): the VGPRs live into each
basic block (backward dataflow over the block graph), so the loop-carried registers of the
lane loop can be counted and compared before and after a change.

    python tools/isa_live.py LISTING.s [BLOCK ...]   (default block: the SC_ITER header)

An instruction's first VGPR operand is its definition when the opcode writes a VGPR (VALU
other than v_cmp*/v_readfirstlane/v_readlane, loads, ds_read*, ds_bpermute); every other
VGPR operand is a use. Register ranges v[a:b] count each register."""
import re
import sys


def regs(tok):
    m = re.match(r"v\[(\d+):(\d+)\]", tok)
    if m:
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", tok)
    return [int(m.group(1))] if m else []


def parse(path):
    blocks, order, cur, infn = {}, [], None, False
    for ln in open(path):
        s = ln.strip()
        if re.match(r"^_ZN2fr12trace_kernel\S*:", s):
            infn = True
            cur = "entry"
            blocks[cur] = {"ins": [], "mark": None}
            order.append(cur)
            continue
        if not infn:
            continue
        if s.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\d+_\d+):|^; (%bb\.\d+):", s)
        if m:
            cur = m.group(1) or m.group(2)
            blocks[cur] = {"ins": [], "mark": None}
            order.append(cur)
            continue
        m = re.search(r";FRSEC (\w+)", s)
        if m:
            blocks[cur]["mark"] = m.group(1)
        if not s or s.startswith(";") or s.startswith("."):
            continue
        blocks[cur]["ins"].append(s.split(";")[0])
    return blocks, order


def use_def(ins):
    parts = ins.replace(",", " ").split()
    op, ops = parts[0], parts[1:]
    vr = [regs(t.lstrip("-|").rstrip("|")) for t in ops]
    defs, uses = set(), set()
    writes = (op.startswith("v_") and not op.startswith("v_cmp") and not op.startswith("v_readfirstlane")
              and not op.startswith("v_readlane")) or op.startswith("global_load") or op.startswith(
        "buffer_load") or op.startswith("ds_read") or op.startswith("ds_bpermute") or op.startswith("flat_load") \
        or op.startswith("scratch_load")
    if writes and vr and vr[0]:
        defs = set(vr[0])
        rest = vr[1:]
        if op.startswith("v_fmac") or op.startswith("v_mac"):
            uses |= set(vr[0])
    else:
        rest = vr
    for r in rest:
        uses |= set(r)
    return op, uses, defs


def succs(blocks, order):
    out = {}
    for i, b in enumerate(order):
        ins = blocks[b]["ins"]
        tgt = []
        last = ins[-1] if ins else ""
        for x in ins:
            if x.startswith("s_cbranch") or x.startswith("s_branch"):
                tgt.append(x.split()[1])
        if not last.startswith("s_branch") and not last.startswith("s_endpgm") and i + 1 < len(order):
            tgt.append(order[i + 1])
        out[b] = [t for t in tgt if t in blocks]
    return out


def live_in(blocks, order):
    sc = succs(blocks, order)
    ud = {}
    for b in order:
        use, dfn = set(), set()
        for ins in blocks[b]["ins"]:
            _, u, d = use_def(ins)
            use |= (u - dfn)
            dfn |= d
        ud[b] = (use, dfn)
    lin = {b: set() for b in order}
    changed = True
    while changed:
        changed = False
        for b in reversed(order):
            lout = set()
            for s in sc[b]:
                lout |= lin[s]
            new = ud[b][0] | (lout - ud[b][1])
            if new != lin[b]:
                lin[b] = new
                changed = True
    return lin


if __name__ == "__main__":
    blocks, order = parse(sys.argv[1])
    lin = live_in(blocks, order)
    names = sys.argv[2:] or [b for b in order if blocks[b]["mark"] == "SC_ITER"]
    for b in names:
        print(b, blocks[b]["mark"], len(lin[b]), sorted(lin[b]))
    print("max live-in over blocks:", max(len(v) for v in lin.values()))
