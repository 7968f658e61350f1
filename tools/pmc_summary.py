"""Summarise a tools/profile.sh run: per-launch PMC values of trace_kernel and the
kernel-trace statistics.

    python tools/pmc_summary.py gpurun_out/prof/<tag> [--write profiles/pmc_trace_kernel.json]
    python tools/pmc_summary.py --runs DIR... [--segments N]   (one rocprofv3 --pmc run per DIR,
        each with --kernel-trace --stats: counters averaged over the trace_kernel launches, the
        launch time from the runs' warm launches, VALU lane-slots per segment when N is given)

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


def runs_summary(dirs, segments=None):
    out = collections.defaultdict(list)
    warm_ns = []
    for dpath in dirs:
        for f in glob.glob(os.path.join(dpath, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if "trace_kernel" in r["Kernel_Name"]:
                    out[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for f in glob.glob(os.path.join(dpath, "**", "*kernel_trace.csv"), recursive=True):
            ts = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in csv.DictReader(open(f))
                        if "trace_kernel" in r["Kernel_Name"])
            warm_ns += [e - s for s, e in ts[1:]]  # the first (cold) launch of each run set aside
    res = {k: sum(v) / len(v) for k, v in out.items()}
    res["launches_per_counter"] = {k: len(v) for k, v in out.items()}
    ns = sum(warm_ns) / len(warm_ns) if warm_ns else None
    res["warm_launch_ns_under_counters"] = ns
    if ns and "SQ_INSTS_VALU" in res and "GRBM_GUI_ACTIVE" in res:
        clk = res["GRBM_GUI_ACTIVE"] / 8 / (ns * 1e-9)
        res["clock_ghz"] = clk / 1e9
        res["valu_issue_frac"] = res["SQ_INSTS_VALU"] / (ns * 1e-9) / (1024 * clk / 2)
    if "SQ_WAIT_ANY" in res and "SQ_WAVE_CYCLES" in res:
        res["wait_any_over_wave_cycles"] = res["SQ_WAIT_ANY"] / res["SQ_WAVE_CYCLES"]
    if "WRITE_SIZE" in res:
        res["write_bytes"] = res["WRITE_SIZE"] * 1024
    if "FETCH_SIZE" in res:
        res["fetch_bytes_x2"] = 2 * res["FETCH_SIZE"] * 1024
    if segments and "SQ_INSTS_VALU" in res:
        res["segments"] = segments
        res["valu_lane_slots_per_segment"] = res["SQ_INSTS_VALU"] * 64 / segments
    return res


def main():
    if sys.argv[1] == "--runs":
        args = sys.argv[2:]
        seg = None
        if "--segments" in args:
            seg = float(args[args.index("--segments") + 1])
            args = args[:args.index("--segments")] + args[args.index("--segments") + 2:]
        print(json.dumps(runs_summary(args, seg), indent=1))
        return
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
