"""Static instruction mix of the C2 frame kernel between its phase marks (diagnostics).

Compiles render.hip for gfx950 with -DERAY_ISA_MARKS (each ERAY_TRACE point becomes an asm
comment) and counts instruction classes between consecutive marks, in code order.
"""
import collections
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from eray_amd import build as B  # noqa: E402

KERNEL = sys.argv[1] if len(sys.argv) > 1 else "frame_kernelILb1ELb0ELi0ELb1E"
out = "/tmp/eray_isa_marks.s"
flags = [f for f in B.CXXFLAGS if f != "-fPIC"]
subprocess.run([B.hipcc(), *flags, "-DERAY_ISA_MARKS", "--cuda-device-only", "-S",
                os.path.join(B.CSRC, "render.hip"), "-o", out], check=True, capture_output=True)
lines = open(out).read().split("\n")
start = next(i for i, l in enumerate(lines) if l.startswith("_Z") and KERNEL in l.split(":")[0])
end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
seg, counts = "start", collections.OrderedDict()
for l in lines[start:end]:
    m = re.search(r"ERAY_MARK (\d+)", l)
    if m:
        seg = f"->{m.group(1)}@{len(counts)}"
        continue
    t = l.strip()
    if not t or t.startswith((";", ".")) or t.endswith(":"):
        continue
    op = t.split()[0]
    cls = ("valu" if op.startswith("v_") else "salu" if op.startswith("s_") and not op.startswith(("s_load", "s_buffer", "s_waitcnt", "s_cbranch", "s_branch", "s_memtime", "s_memrealtime", "s_nop"))
           else "smem" if op.startswith(("s_load", "s_buffer")) else "wait" if op.startswith("s_waitcnt")
           else "branch" if op.startswith(("s_cbranch", "s_branch")) else "nop" if op.startswith("s_nop")
           else "lds" if op.startswith("ds_") else "vmem" if op.startswith(("global_", "buffer_", "scratch_", "flat_")) else "other")
    counts.setdefault(seg, collections.Counter())[cls] += 1
tot = collections.Counter()
for seg, c in counts.items():
    tot += c
    print(f"{seg:12s} " + " ".join(f"{k}={c[k]}" for k in ("valu", "salu", "smem", "lds", "vmem", "wait", "branch", "nop", "other")))
print("total       ", dict(tot))
