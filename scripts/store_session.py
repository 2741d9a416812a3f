"""Copies a measurement session's results (scripts/r02_session.sh, gpurun_out/) into
profiles/<round>/: the C2 bench line, its rocprofv3 kernel statistics, the PMC traffic summaries
per configuration, the other configurations' lines and the multi-rank rehearsals.

    python scripts/store_session.py r02
"""
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def last_json(path):
    lines = [x for x in open(path) if x.startswith("{")]
    return json.loads(lines[-1]) if lines else None


def main(tag: str) -> None:
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(os.path.join(dst, "configs"), exist_ok=True)
    d = last_json(os.path.join(OUT, "bench.log"))
    if d:
        with open(os.path.join(dst, "bench_c2.json"), "w") as f:
            json.dump(d, f, indent=1)
    stats = glob.glob(os.path.join(OUT, "prof", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(dst, "kernel_stats_c2.csv"))
    for name in ("c2", "c3", "ns_4k_70k", "c5_1gpu"):
        if os.path.isdir(os.path.join(OUT, f"pmc_{name}")):
            subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_traffic.py"), tag, f"pmc_{name}",
                            os.path.join(tag, f"pmc_traffic_{name}.json")], check=True)
    for path in glob.glob(os.path.join(OUT, "cfg_*.log")) + glob.glob(os.path.join(OUT, "rehearsal_n*.log")):
        d = last_json(path)
        if d:
            name = os.path.basename(path)[:-4].replace("cfg_", "")
            with open(os.path.join(dst, "configs", name + ".json"), "w") as f:
                json.dump(d, f, indent=1)
    print("stored into", os.path.relpath(dst, ROOT))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02")
