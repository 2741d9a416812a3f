#!/bin/bash
# A/B of the static C3 frame across builds of earlier commits copied to ab_<name>/ (not tracked).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out /tmp/eray_meshes
M=/tmp/eray_meshes
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o $M/standin70k.obj > /dev/null || exit 1
for rep in 1 2; do
for t in ${AB_TREES:-head r01}; do
  if [ $t = head ]; then D=.; else D=ab_$t; fi
  X=""; grep -q no-moving-camera $D/bench.py && X="--no-moving-camera"
  (cd $D && timeout -k 10 200 python bench.py --mesh $M/standin70k.obj --steps 400 --warmup 40 --no-cpu-baseline $X > $GRAFT_REPO_ROOT/gpurun_out/ab_c3_${t}_$rep.log 2>&1) || exit 1
  python - "$t" "$rep" <<'PY'
import json,sys
l=[x for x in open(f"gpurun_out/ab_c3_{sys.argv[1]}_{sys.argv[2]}.log") if x.startswith("{")][-1]
d=json.loads(l); print(sys.argv[1], sys.argv[2], d["frame_ms"], d["render_kernel_ms"])
PY
done; done
