"""Per-launch counter values of trace_kernel from a tools/pmc_mix.sh run:
    python tools/mix_summary.py gpurun_out/prof/<TAG>"""
import collections
import csv
import glob
import json
import os
import sys

vals = collections.defaultdict(list)
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "trace_kernel" in r["Kernel_Name"]:
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (_, name), v in per.items():
        vals[name].append(v)
out = {k: sum(v) / len(v) for k, v in sorted(vals.items())}
valu = out.get("SQ_INSTS_VALU")
if valu:
    for k in ("SQ_INSTS_VALU_ADD_F32", "SQ_INSTS_VALU_MUL_F32", "SQ_INSTS_VALU_FMA_F32", "SQ_INSTS_VALU_TRANS_F32",
              "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_CVT"):
        if k in out:
            out[k + "_frac_of_valu"] = round(out[k] / valu, 4)
print(json.dumps(out, indent=1))
