"""Per-kernel register / spill / occupancy / LDS table of one HIP source (diagnostics, CPU only).

    python scripts/kernel_resources.py eray_amd/csrc/render.hip [--filter frame_kernel] [-D NAME=VAL ...]

Compiles the source for gfx950 with the product's flags (device code only) and the
`-Rpass-analysis=kernel-resource-usage` remarks, then prints one row per kernel.
"""
from __future__ import annotations

import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from eray_amd.build import CXXFLAGS, hipcc  # noqa: E402


def demangle(names: list[str]) -> list[str]:
    try:
        r = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-cxxfilt"], input="\n".join(names), capture_output=True,
                           text=True, check=True)
        return r.stdout.splitlines()
    except (OSError, subprocess.CalledProcessError):
        return names


def resources(src: str, defines: list[str]) -> list[dict]:
    with tempfile.TemporaryDirectory() as tmp:
        lang = [] if src.endswith(".hip") else ["-x", "hip"]
        cmd = [hipcc(), *CXXFLAGS, "-I" + os.path.join(ROOT, "eray_amd", "csrc"), *lang, "--cuda-device-only", "-c", src,
               "-o", os.path.join(tmp, "k.o"), "-Rpass-analysis=kernel-resource-usage", *("-D" + d for d in defines)]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode:
            raise SystemExit(r.stderr[-4000:])
    rows: list[dict] = []
    for line in r.stderr.splitlines():
        m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|SGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                      r"SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]): (\S+)", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            rows.append({"name": v})
        elif rows:
            rows[-1][k.split(" [")[0]] = v
    for row, nm in zip(rows, demangle([r["name"] for r in rows])):
        row["name"] = nm
    return rows


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("source")
    ap.add_argument("--filter", default="")
    ap.add_argument("-D", dest="defines", action="append", default=[])
    a = ap.parse_args()
    for r in resources(a.source, a.defines):
        if a.filter not in r["name"]:
            continue
        name = re.sub(r"\(.*", "", r["name"]).replace("eray::gpu::(anonymous namespace)::", "")
        print(f"{r.get('VGPRs', '?'):>4} vgpr {r.get('VGPRs Spill', '?'):>3} vspill {r.get('SGPRs', '?'):>4} sgpr "
              f"{r.get('SGPRs Spill', '?'):>4} sspill {r.get('ScratchSize', '?'):>5} scratch "
              f"occ {r.get('Occupancy', '?'):>2} lds {r.get('LDS Size', '?'):>6}  {name}")


if __name__ == "__main__":
    main()
