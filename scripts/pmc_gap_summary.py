"""Summarise scripts/fill_gap.sh's rocprofv3 runs (diagnostics): per kernel — the frame kernel's
empty-scene fill and the write ceiling (render.hip ceiling_fill_kernel), both in one process —
the kernel-trace statistics and the median of every collected counter per dispatch.

    python scripts/pmc_gap_summary.py <dir under gpurun_out> <output json> [--round rNN]
"""
from __future__ import annotations

import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    for k in ("ceiling_fill_kernel", "frame_kernel", "fill_kernel"):
        if k in name:
            return k
    return name


def main() -> None:
    src = os.path.join(ROOT, "gpurun_out", sys.argv[1])
    dst = sys.argv[2]
    rnd = sys.argv[sys.argv.index("--round") + 1] if "--round" in sys.argv else None
    out = {"round": rnd, "source": sys.argv[1], "kernels": {}}
    for path in glob.glob(os.path.join(src, "stats", "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            if "frame_kernel" in r["Name"] or "ceiling_fill_kernel" in r["Name"]:
                out["kernels"].setdefault(short(r["Name"]), {})["stats"] = {
                    "calls": int(r["Calls"]), "mean_us": round(float(r["AverageNs"]) / 1e3, 3),
                    "min_us": round(float(r["MinNs"]) / 1e3, 3), "max_us": round(float(r["MaxNs"]) / 1e3, 3)}
    per = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(src, "*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            per[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in per.items():
        out["kernels"].setdefault(k, {})["counters_median_per_dispatch"] = {n: statistics.median(v) for n, v in c.items()}
    with open(dst, "w") as f:
        json.dump(out, f, indent=2)
    print("wrote", dst)


if __name__ == "__main__":
    main()
