"""Per-leg kernel rows of a rocprofv3 run of bench.py (round 4).

    rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d gpurun_out/<dir> -o run \
        -- python3 bench.py ...
    python scripts/prof_legs.py gpurun_out/<dir> profiles/r04/<name>_legs.csv

bench.py wraps each of its legs in a ROCTx range named after the leg and its launch size
(`steps_F8`, `timed_F8`, `latency_F1`, `fill_floor_F8`, `ns_slots4_timed_F1`, ...).  Every leg ends
with a synchronisation before its range closes, so a dispatch belongs to the range whose
[start, end] holds the dispatch's [start, end].  The output has one row per (leg, kernel): calls,
mean / median / min / max duration in microseconds — the rows the bench line's dispatch-timed
kernel figures (eray_time_frames_ring) must reproduce, one launch size per row.
"""
from __future__ import annotations

import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def _find(d: str, suffix: str) -> list[str]:
    return sorted(glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True))


def _short(name: str) -> str:
    """frame_kernel<...> / fill_kernel<...> / other kernels by their base name."""
    base = name.replace("(anonymous namespace)", "")
    for k in ("ceiling_fill_kernel", "frame_kernel", "fill_kernel", "trace_kernel", "trace_binned_kernel", "trace_heavy_kernel",
              "trace_cull_kernel", "camera_setup_kernel", "bin_pairs_kernel", "material_example_kernel"):
        if k in base:
            return k
    return base.split("(")[0].split("<")[0].split("::")[-1].strip() or name[:40]


def ranges(d: str) -> list[tuple[str, int, int]]:
    out = []
    for path in _find(d, "marker_api_trace.csv"):
        with open(path) as f:
            for row in csv.DictReader(f):
                name = row.get("Function") or row.get("Message") or ""
                if not name or name.startswith("roctx"):
                    continue
                out.append((name, int(row["Start_Timestamp"]), int(row["End_Timestamp"])))
    return out


def rows(d: str):
    rs = ranges(d)
    per = defaultdict(list)
    for path in _find(d, "kernel_trace.csv"):
        with open(path) as f:
            for row in csv.DictReader(f):
                s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
                leg = "(outside the ranges)"
                for name, r0, r1 in rs:
                    if r0 <= s and e <= r1:
                        leg = name
                        break
                per[(leg, _short(row["Kernel_Name"]))].append((e - s) / 1e3)
    return per


def main() -> None:
    src, dst = sys.argv[1], sys.argv[2]
    per = rows(src)
    if not per:
        raise SystemExit(f"no kernel_trace.csv under {src}")
    os.makedirs(os.path.dirname(os.path.abspath(dst)), exist_ok=True)
    with open(dst, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["leg", "kernel", "calls", "mean_us", "median_us", "min_us", "max_us"])
        for (leg, k), v in sorted(per.items()):
            w.writerow([leg, k, len(v), round(statistics.mean(v), 3), round(statistics.median(v), 3),
                        round(min(v), 3), round(max(v), 3)])
    print("wrote", dst)


if __name__ == "__main__":
    main()
