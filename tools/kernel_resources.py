"""Per-variant resources of trace_kernel from hipcc's -Rpass-analysis=kernel-resource-usage
remarks: python tools/kernel_resources.py REMARKS_FILE"""
import re
import sys

cur, rows = None, []
for line in open(sys.argv[1]):
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key in ["VGPRs", "TotalSGPRs", r"Occupancy \[waves/SIMD\]", "SGPRs Spill", r"LDS Size \[bytes/block\]"]:
        m = re.search(key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0]] = int(m.group(1))
for r in rows:
    m = re.search(r"trace_kernelILi(\d)ELb(\d)ELi\d+ELi(\d)ELb(\d)ELb(\d)ELi(\d)E", r["name"])
    if m:
        print("KS=%s HP=%s MAXD=%s BVH=%s MT=%s DEFER=%s" % m.groups(), "VGPR", r.get("VGPRs"), "SGPR",
              r.get("TotalSGPRs"), "occ", r.get("Occupancy"), "spill", r.get("SGPRs"))
