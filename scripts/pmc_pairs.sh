#!/bin/bash
# Counter passes over the bins chain of C5's moving-camera loop (bin_pairs / scatter / setup),
# each pass its own run; plus the bin statistics of the scene camera.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=${OUT:-gpurun_out/pmcp}
mkdir -p $OUT /tmp/eray_meshes
export TMPDIR=/tmp
python -m eray_amd.meshgen --triangles 1000000 --seed 1234 -o /tmp/eray_meshes/synth1m.obj > /dev/null || exit 1
timeout -k 10 120 python scripts/bin_stats.py /tmp/eray_meshes/synth1m.obj 7680 4320 > $OUT/bin_stats.txt 2>&1 || { tail $OUT/bin_stats.txt; exit 1; }
cat $OUT/bin_stats.txt
pass() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-include-regex 'bin_pairs|bin_scatter|camera_setup' --output-format csv \
      -d $OUT/$name -o $name -- python scripts/moving_camera.py --mesh /tmp/eray_meshes/synth1m.obj --width 7680 --height 4320 --frames 8 > $OUT/$name.log 2>&1
  local rc=$?
  echo "=== pmc $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -20 $OUT/$name.log; exit $rc; fi
}
pass a SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS
pass b SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES
python - $OUT <<'PY'
import csv, glob, sys, collections, re
d = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(\w+)(<[^>]*>)?\(", r["Kernel_Name"].replace("(anonymous namespace)", ""))
        k = (m.group(1) + (m.group(2) or "")) if m else r["Kernel_Name"][:40]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(k, {c: round(sum(v) / max(len(v), 1)) for c, v in sorted(cs.items())})
PY
