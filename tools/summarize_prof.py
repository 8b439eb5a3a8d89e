"""Condense rocprofv3 CSV output into small committed summaries (profiles/<name>/).

    python tools/summarize_prof.py <rocprof_dir> <out_dir>

Copies ``*_kernel_stats.csv`` (names shortened) and, when a ``*_counter_collection.csv`` is present,
writes ``pmc_summary.csv``: per kernel, the sum of each raw counter over all dispatches."""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    depth = 0
    for i, ch in enumerate(name):  # cut the argument list (first '(' outside template brackets)
        depth += ch == "<"
        depth -= ch == ">"
        if ch == "(" and depth == 0 and i > 0:
            name = name[:i]
            break
    return name[:120]


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    for p in glob.glob(os.path.join(src, "*_kernel_stats.csv")):
        rows = list(csv.DictReader(open(p)))
        with open(os.path.join(dst, "kernel_stats.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "calls", "total_ms", "avg_us", "pct"])
            for r in rows:
                w.writerow([short(r["Name"]), r["Calls"], "%.3f" % (float(r["TotalDurationNs"]) / 1e6),
                            "%.2f" % (float(r["AverageNs"]) / 1e3), r["Percentage"]])
    for p in glob.glob(os.path.join(src, "*_counter_collection.csv")):
        agg = defaultdict(lambda: defaultdict(float))
        disp = defaultdict(set)
        for r in csv.DictReader(open(p)):
            k = short(r["Kernel_Name"])
            agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
        counters = sorted({c for v in agg.values() for c in v})
        with open(os.path.join(dst, "pmc_summary.csv"), "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "dispatches"] + counters)
            for k, v in sorted(agg.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0)):
                w.writerow([k, len(disp[k])] + ["%.0f" % v.get(c, 0.0) for c in counters])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
