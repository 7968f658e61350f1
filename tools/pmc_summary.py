"""Summarise a tools/profile.sh run: per-launch PMC values of trace_kernel and the
kernel-trace statistics.

    python tools/pmc_summary.py gpurun_out/prof/<tag> [--write profiles/pmc_trace_kernel.json]

--write stores the per-launch HBM bytes that bench.py reports as roofline.traffic."""
import collections
import csv
import glob
import json
import os
import sys


def load(dirpath):
    out = collections.defaultdict(list)
    for f in glob.glob(os.path.join(dirpath, "pmc_*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if "trace_kernel" in r["Kernel_Name"]:
                out[r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {k: sum(v) / len(v) for k, v in out.items()}
    stats = os.path.join(dirpath, "trace", "trace_kernel_stats.csv")
    if os.path.exists(stats):
        for r in csv.DictReader(open(stats)):
            if "trace_kernel" in r["Name"]:
                res["avg_ns"] = float(r["AverageNs"])
                res["calls"] = int(r["Calls"])
    return res


def main():
    d = load(sys.argv[1])
    hbm = None
    ns = d.get("avg_ns", 0)
    print(json.dumps(d, indent=1))
    if ns and "SQ_INSTS_VALU" in d:
        clk = d.get("GRBM_GUI_ACTIVE", 0) / 8 / (ns * 1e-9) / 1e9 if "GRBM_GUI_ACTIVE" in d else 2.1
        peak = 1024 * clk * 1e9 / 2  # wave-instructions/s: 1024 SIMDs, 2 cycles per wave64 VALU op
        print(f"clock ~{clk:.2f} GHz; VALU issue {d['SQ_INSTS_VALU'] / (ns * 1e-9) / peak:.1%} of peak")
    if ns and "FETCH_SIZE" in d:
        # gfx950: FETCH_SIZE (KB) counts 64 B per 128-B request: double it (MI355X_MICROARCH.md §HBM)
        hbm = (2 * d["FETCH_SIZE"] + d.get("WRITE_SIZE", 0)) * 1024
        print(f"HBM bytes/launch ~{hbm:.3e} ({hbm / (ns * 1e-9) / 1e9:.2f} GB/s)")
    if "--write" in sys.argv and hbm is not None:
        path = sys.argv[sys.argv.index("--write") + 1]
        rec = {"workload": "scene_08 1920x1080 256spp d8", "kernel": "trace_kernel",
               "hbm_bytes_per_launch": round(hbm), "fetch_size_kb": d["FETCH_SIZE"],
               "write_size_kb": d.get("WRITE_SIZE"), "avg_ns": ns, "source": sys.argv[1],
               "note": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes; FETCH_SIZE doubled "
                       "(gfx950, MI355X_MICROARCH.md HBM section); WRITE_SIZE as reported (uncalibrated for "
                       "12-B scattered stores)"}
        with open(path, "w") as f:
            json.dump(rec, f, indent=1)
        print("wrote", path)


if __name__ == "__main__":
    main()
