"""Warm per-launch kernel times from a counter-free `rocprofv3 --kernel-trace` run.

    python tools/ktrace_summary.py DIR [--skip N] [--last K] [--match trace_kernel] [--out FILE]

DIR holds rocprofv3's `*kernel_trace.csv` (any depth). Launches of each kernel whose name
contains one of the --match strings are ordered by start time; the first --skip of them
(the cold launch and the warm-up frames) are listed apart, and the mean, min, max and
standard deviation are over the rest (or the last --last K of them). rocprofv3's own
`--stats` average includes the cold launch; this is the figure to set beside the bench
line's HIP-event mean."""
import argparse
import csv
import glob
import json
import os
import statistics


def load(dirpath, matches):
    rows = {}
    for f in glob.glob(os.path.join(dirpath, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            if not any(m in name for m in matches):
                continue
            short = name.split("(")[0].split("<")[0].strip() or name
            tmpl = name[len(short):].split("(")[0] if "<" in name else ""
            key = short + (tmpl[:80] if tmpl else "")
            rows.setdefault(key, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return rows


def summarise(launches, skip, last):
    launches = sorted(launches)
    ms = [(e - s) / 1e6 for s, e in launches]
    cold, warm = ms[:skip], ms[skip:]
    if last:
        warm = warm[-last:]
    out = {"launches": len(ms), "skipped_ms": [round(x, 4) for x in cold], "n": len(warm)}
    if warm:
        out.update({"mean_ms": round(statistics.fmean(warm), 4), "min_ms": round(min(warm), 4),
                    "max_ms": round(max(warm), 4),
                    "std_ms": round(statistics.pstdev(warm), 4) if len(warm) > 1 else 0.0,
                    "all_launches_mean_ms": round(statistics.fmean(ms), 4)})
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--skip", type=int, default=1)
    ap.add_argument("--last", type=int, default=0)
    ap.add_argument("--match", action="append", default=None)
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = load(a.dir, a.match or ["trace_kernel", "sum_"])
    res = {"source": a.dir, "skip": a.skip, "last": a.last or None,
           "kernels": {k: summarise(v, a.skip, a.last) for k, v in sorted(rows.items())}}
    text = json.dumps(res, indent=1)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
