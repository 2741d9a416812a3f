"""Summarise scripts/mat_pmc.sh's rocprofv3 runs of material_example_kernel into profiles/:
the kernel-trace statistics (copied) and per-dispatch counters with the derived figures —
achieved write bandwidth from the kernel's own average duration (16 B written per texel), the
share of wave cycles spent waiting (SQ_WAIT_ANY / SQ_WAVE_CYCLES), VALU instructions per texel
and WRITE_SIZE bytes against the algorithmic 16 B per texel.

    python scripts/mat_pmc_summary.py r05 [pmc dir under gpurun_out, default mat_pmc]"""
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
TEXELS = 1024 * 1024  # scripts/ab_probe.py mat: main.rs's 1024 x 1024 texture
PEAK_GBS = 8000.0


def main() -> None:
    tag = sys.argv[1] if len(sys.argv) > 1 else "r05"
    d = sys.argv[2] if len(sys.argv) > 2 else "mat_pmc"
    os.makedirs(os.path.join(PROF, tag), exist_ok=True)
    stats = glob.glob(os.path.join(OUT, d, "stats", "**", "*kernel_stats.csv"), recursive=True)
    avg_ns = None
    if stats:
        with open(stats[0]) as f:
            rows = list(csv.DictReader(f))
        with open(os.path.join(PROF, tag, "material_kernel_stats.csv"), "w") as f:
            f.write(open(stats[0]).read())
        for r in rows:
            if "material_example_kernel" in r["Name"]:
                avg_ns = float(r["AverageNs"])
    per = defaultdict(list)
    for path in glob.glob(os.path.join(OUT, d, "*", "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for row in csv.DictReader(f):
                if "material_example_kernel" in row["Kernel_Name"]:
                    per[row["Counter_Name"]].append(float(row["Counter_Value"]))
    c = {k: statistics.median(v) for k, v in per.items()}
    out = {"round": tag, "kernel": "material_example_kernel (eray_amd/csrc/shaderlib.hip)", "texels": TEXELS,
           "algorithmic_bytes": TEXELS * 16, "counters_median_per_dispatch": c}
    if avg_ns:
        gbs = TEXELS * 16 / avg_ns
        out.update(avg_duration_us=round(avg_ns / 1e3, 3), achieved_gbs=round(gbs, 1), frac=round(gbs / PEAK_GBS, 4))
    if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
        out["wait_frac"] = round(c.get("SQ_WAIT_ANY", 0.0) / c["SQ_WAVE_CYCLES"], 4)
    if "SQ_INSTS_VALU" in c:
        out["valu_insts_per_texel"] = round(c["SQ_INSTS_VALU"] * 64 / TEXELS, 2)  # (per wave -> per lane)
    f64 = sum(c.get(k, 0.0) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64"))
    if f64 and c.get("SQ_INSTS_VALU"):
        out["fp64_share_of_valu"] = round(f64 / c["SQ_INSTS_VALU"], 4)
    if avg_ns and c.get("SQ_INST_CYCLES_VALU"):
        # VALU issue cycles over every SIMD's cycles of the kernel (1024 SIMDs at 2.4 GHz): the
        # fraction of the chip's VALU issue the kernel used
        out["valu_issue_frac"] = round(c["SQ_INST_CYCLES_VALU"] / (1024 * avg_ns * 2.4), 4)
    if "WRITE_SIZE" in c:
        out["write_bytes"] = c["WRITE_SIZE"] * 1024
        out["write_over_algorithmic"] = round(c["WRITE_SIZE"] * 1024 / (TEXELS * 16), 4)
    path = os.path.join(PROF, tag, "material_pmc.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=2)
    print("wrote", os.path.relpath(path, ROOT), json.dumps({k: v for k, v in out.items() if k != "counters_median_per_dispatch"}))


if __name__ == "__main__":
    main()
