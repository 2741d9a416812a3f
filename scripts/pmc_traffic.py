"""Summarise a rocprofv3 session of bench.py into profiles/ (run after scripts/gpu_session.sh and
scripts/gpu_pmc.sh have filled gpurun_out/).

  * profiles/<round>_kernel_stats.csv   per-kernel count / total / average duration (the
                                         rocprofv3 --kernel-trace --stats database)
  * profiles/pmc_traffic.json           frame-kernel counters per launch; HBM bytes per launch =
                                         2 x FETCH_SIZE + WRITE_SIZE (KB), the gfx950 correction of
                                         MI355X_MICROARCH.md (FETCH_SIZE counts half the bytes of
                                         wide streaming reads; WRITE_SIZE is exact for 16-B stores)
"""
import csv
import glob
import json
import os
import sqlite3
import statistics
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")
PROF = os.path.join(ROOT, "profiles")


def kernel_stats(tag: str) -> None:
    dbs = glob.glob(os.path.join(OUT, "prof", "**", "*results.db"), recursive=True)
    if not dbs:
        print("no rocprofv3 stats database under gpurun_out/prof", file=sys.stderr)
        return
    con = sqlite3.connect(dbs[0])
    cur = con.execute("select * from top_kernels")
    cols = [d[0] for d in cur.description]
    path = os.path.join(PROF, f"{tag}_kernel_stats.csv")
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(cols)
        for row in cur:
            w.writerow(row)
    print("wrote", os.path.relpath(path, ROOT))


def pmc(tag: str) -> None:
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values per dispatch
    for path in glob.glob(os.path.join(OUT, "pmc", "*", "*counter_collection.csv")):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                if "frame_kernel" not in name:
                    continue
                per[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    if not per:
        print("no frame_kernel counters under gpurun_out/pmc", file=sys.stderr)
        return
    name = max(per, key=lambda k: len(per[k].get("WRITE_SIZE", [])))
    c = {k: statistics.mean(v) for k, v in per[name].items()}
    fetch, write = c.get("FETCH_SIZE", 0.0) * 1024, c.get("WRITE_SIZE", 0.0) * 1024
    out = {"round": tag, "frame_kernel": {
        "kernel": name,
        "dispatches": len(per[name].get("WRITE_SIZE", [])),
        "counters_mean_per_dispatch": c,
        "fetch_bytes_corrected": 2 * fetch,
        "write_bytes": write,
        "hbm_bytes_per_launch": int(2 * fetch + write),
    }}
    path = os.path.join(PROF, "pmc_traffic.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=2)
    print("wrote", os.path.relpath(path, ROOT), out["frame_kernel"]["hbm_bytes_per_launch"])


if __name__ == "__main__":
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    os.makedirs(PROF, exist_ok=True)
    kernel_stats(tag)
    pmc(tag)
