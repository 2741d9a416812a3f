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
    csvs = glob.glob(os.path.join(OUT, "prof", "**", "*kernel_stats.csv"), recursive=True)
    path = os.path.join(PROF, f"{tag}_kernel_stats.csv")
    if csvs:  # rocprofv3 --output-format csv
        with open(csvs[0]) as src, open(path, "w") as dst:
            dst.write(src.read())
        print("wrote", os.path.relpath(path, ROOT))
        return
    dbs = glob.glob(os.path.join(OUT, "prof", "**", "*results.db"), recursive=True)
    if not dbs:
        print("no rocprofv3 stats under gpurun_out/prof", file=sys.stderr)
        return
    con = sqlite3.connect(dbs[0])
    cur = con.execute("select * from top_kernels")
    cols = [d[0] for d in cur.description]
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(cols)
        for row in cur:
            w.writerow(row)
    print("wrote", os.path.relpath(path, ROOT))


def pmc(tag: str, pmc_dir: str = "pmc", out_name: str = "pmc_traffic.json", workload=None) -> None:
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> values per dispatch
    for path in glob.glob(os.path.join(OUT, pmc_dir, "*", "*counter_collection.csv")):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                if "frame_kernel" not in name and "fill_kernel" not in name:
                    continue
                per[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    if not per:
        print("no frame_kernel counters under gpurun_out/pmc", file=sys.stderr)
        return
    frames = [k for k in per if "frame_kernel" in k]
    name = max(frames, key=lambda k: len(per[k].get("WRITE_SIZE", [])))
    # the median dispatch: the bench's measured launches (frames in flight) outnumber its one
    # instrumented single-frame render
    c = {k: statistics.median(v) for k, v in per[name].items()}
    dispatches = len(per[name].get("WRITE_SIZE", []))
    fetch, write = c.get("FETCH_SIZE", 0.0) * 1024, c.get("WRITE_SIZE", 0.0) * 1024
    # frames whose background comes from the separate fill_kernel (dense large-mesh builds): one
    # fill launch per frame launch, its bytes belong to the frame
    # (the separate fill kernel beside a dense frame kernel; not the write ceiling's stream)
    fills = [k for k in per if "fill_kernel" in k and "ceiling_fill_kernel" not in k]
    if fills:
        f = {k: statistics.median(v) for k, v in per[fills[0]].items()}
        fetch += f.get("FETCH_SIZE", 0.0) * 1024
        write += f.get("WRITE_SIZE", 0.0) * 1024
        name = name + " + " + fills[0]
    if workload is None:  # the bench line of the counted run (its JSON line in the pass logs)
        for log in glob.glob(os.path.join(OUT, pmc_dir, "*.log")):
            for line in open(log):
                if line.startswith("{"):
                    d = json.loads(line)
                    cfg = d["config"]
                    workload = {"mesh": cfg["mesh"], "frame": cfg["frame"], "rows_per_gpu": cfg["rows_per_gpu"],
                                "n_gpus": d["n_gpus"], "brute_force": not cfg["culling"],
                                "frames_per_launch": cfg.get("frames_per_launch", 1)}
    out = {"round": tag, "workload": workload, "frame_kernel": {
        "kernel": name,
        "dispatches": dispatches,
        "counters_mean_per_dispatch": c,
        "fetch_bytes_corrected": 2 * fetch,
        "write_bytes": write,
        "hbm_bytes_per_launch": int(2 * fetch + write),
    }}
    path = os.path.join(PROF, out_name)
    with open(path, "w") as f:
        json.dump(out, f, indent=2)
    print("wrote", os.path.relpath(path, ROOT), out["frame_kernel"]["hbm_bytes_per_launch"])


if __name__ == "__main__":
    # usage: pmc_traffic.py [tag] [pmc dir under gpurun_out] [output file name under profiles/]
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    os.makedirs(PROF, exist_ok=True)
    if len(sys.argv) > 2:
        pmc(tag, sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else f"pmc_traffic_{sys.argv[2]}.json")
    else:
        kernel_stats(tag)
        pmc(tag)
