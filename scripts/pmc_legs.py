"""Frame-kernel counter summaries per workload (round 4), from rocprofv3 --pmc passes of bench.py.

    python scripts/pmc_legs.py <pass dir under gpurun_out> <output json> [--north-star SLOTS]
                                                                        [--workload JSON] [--round rNN]

Each pass directory holds one rocprofv3 counter run per counter group (scripts/gpu_pmc.sh:
`sq`, `fetch`, `write`, each its own run, kernel trace only).  Per counter the median over the
dispatches of the frame kernel instantiation with the most dispatches (the bench's measured
launches of one launch size outnumber its one instrumented frame; in a north_star run the
empty-scene fill floor is another instantiation), plus the separate fill kernel's when the launch
shape has one.  HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB counts; the gfx950
correction of MI355X_MICROARCH.md).  The "workload" key is the one bench.py's pmc_record() looks
for: the C2 line's config, or with --north-star the north_star variant of that many ring slots.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import statistics
import sys
from collections import defaultdict


def main() -> None:
    src, dst = sys.argv[1], sys.argv[2]
    ns_slots = int(sys.argv[sys.argv.index("--north-star") + 1]) if "--north-star" in sys.argv else None
    per = defaultdict(lambda: defaultdict(list))
    for path in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"]
                if ("frame_kernel" in name or "fill_kernel" in name) and "ceiling_fill_kernel" not in name:
                    per[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    if not per:
        raise SystemExit(f"no frame_kernel counters under {src}")
    frames = [k for k in per if "frame_kernel" in k]
    name = max(frames, key=lambda k: max(len(v) for v in per[k].values()))
    c = {k: statistics.median(v) for k, v in per[name].items()}
    dispatches = max(len(v) for v in per[name].values())
    fetch, write = c.get("FETCH_SIZE", 0.0) * 1024, c.get("WRITE_SIZE", 0.0) * 1024
    # (the separate fill kernel beside a dense frame kernel; not the write ceiling's stream)
    fills = [k for k in per if "fill_kernel" in k and "ceiling_fill_kernel" not in k]
    if fills:
        f = {k: statistics.median(v) for k, v in per[fills[0]].items()}
        fetch += f.get("FETCH_SIZE", 0.0) * 1024
        write += f.get("WRITE_SIZE", 0.0) * 1024
        name += " + " + fills[0]
    workload = json.loads(sys.argv[sys.argv.index("--workload") + 1]) if "--workload" in sys.argv else None
    for log in ([] if workload else glob.glob(os.path.join(src, "*.log"))):
        for line in open(log):
            if not line.startswith("{"):
                continue
            d = json.loads(line)
            if ns_slots is not None:
                ns = d["north_star"]
                workload = {"mesh": f"meshgen {ns['triangles']} faces seed 42", "frame": ns["frame"],
                            "rows_per_gpu": ns["frame"][1], "n_gpus": 1, "brute_force": False,
                            "frames_per_launch": 1, "ring_slots": ns_slots}
            else:
                cfg = d["config"]
                workload = {"mesh": cfg["mesh"], "frame": cfg["frame"], "rows_per_gpu": cfg["rows_per_gpu"],
                            "n_gpus": d["n_gpus"], "brute_force": not cfg["culling"],
                            "frames_per_launch": cfg.get("frames_per_launch", 1)}
    # the round the summary belongs to: --round, else the profiles/rNN/ directory it is written into
    m = re.search(r"(?:^|/)(r\d\d)(?:/|$)", os.path.abspath(dst))
    rnd = sys.argv[sys.argv.index("--round") + 1] if "--round" in sys.argv else (m.group(1) if m else None)
    out = {"round": rnd, "workload": workload, "frame_kernel": {
        "kernel": name,
        "dispatches": dispatches,
        "counters_mean_per_dispatch": c,
        "fetch_bytes_corrected": 2 * fetch,
        "write_bytes": write,
        "hbm_bytes_per_launch": int(2 * fetch + write),
    }}
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    with open(dst, "w") as f:
        json.dump(out, f, indent=2)
    print("wrote", dst, out["frame_kernel"]["hbm_bytes_per_launch"])


if __name__ == "__main__":
    main()
