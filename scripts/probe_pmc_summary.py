"""Summarise scripts/probe_pmc.sh's rocprofv3 runs of one ab_probe configuration into profiles/:
the kernel-trace statistics (copied) and the frame kernel's per-dispatch counters (median over
dispatches) with the derived figures — HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (the
gfx950 correction of MI355X_MICROARCH.md), the share of wave cycles waiting
(SQ_WAIT_ANY / SQ_WAVE_CYCLES) and the average kernel duration from the statistics.

    python scripts/probe_pmc_summary.py r05 pmc_c5s3 [output name, default <dir>.json]"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def main() -> None:
    tag, d = sys.argv[1], sys.argv[2]
    name = sys.argv[3] if len(sys.argv) > 3 else f"{d}.json"
    os.makedirs(os.path.join(PROF, tag), exist_ok=True)
    out = {"round": tag, "probe": d}
    stats = glob.glob(os.path.join(OUT, d, "stats", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        rows = list(csv.DictReader(open(stats[0])))
        with open(os.path.join(PROF, tag, name.replace(".json", "_kernel_stats.csv")), "w") as f:
            f.write(open(stats[0]).read())
        out["kernels_avg_us"] = {r["Name"][:120]: round(float(r["AverageNs"]) / 1e3, 3) for r in rows}
    per = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(OUT, d, "*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(path)):
            k = "fill_kernel" if "fill_kernel" in row["Kernel_Name"] else "frame_kernel"
            per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for k, cs in per.items():
        c = {n: statistics.median(v) for n, v in cs.items()}
        rec = {"counters_median_per_dispatch": c}
        if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
            rec["hbm_bytes_per_launch"] = int(2 * c.get("FETCH_SIZE", 0.0) * 1024 + c.get("WRITE_SIZE", 0.0) * 1024)
        if c.get("SQ_WAVE_CYCLES"):
            rec["wait_frac"] = round(c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"], 4)
        out[k] = rec
    path = os.path.join(PROF, tag, name)
    with open(path, "w") as f:
        json.dump(out, f, indent=2)
    print("wrote", os.path.relpath(path, ROOT))


if __name__ == "__main__":
    main()
