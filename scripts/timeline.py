"""Diagnostics: the last N kernels of a rocprofv3 kernel trace (csv) — start offset, duration, queue."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
rows = rows[-n:]
t0 = int(rows[0]["Start_Timestamp"])


def short(name):
    name = name.replace("void ", "")
    depth, out = 0, ""
    for ch in name:  # drop template arguments and parameter lists
        if ch in "<(":
            depth += 1
        elif ch in ">)":
            depth -= 1
        elif depth == 0:
            out += ch
    return out.split("::")[-1][:48]


for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:9.2f} {(e - s) / 1e3:8.2f}  q{r.get('Queue_Id', '?'):>3}  {short(r['Kernel_Name'])}")
