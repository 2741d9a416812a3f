#!/bin/bash
# A/B of one configuration's static frame across HEAD and builds of earlier commits in ab_<name>/
# (AB_TREES, AB_ARGS: bench.py arguments; meshes generated under /tmp/eray_meshes).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out /tmp/eray_meshes
M=/tmp/eray_meshes
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o $M/standin70k.obj > /dev/null || exit 1
[ "${AB_C5:-0}" = 1 ] && { python -m eray_amd.meshgen --triangles 1000000 --seed 1234 -o $M/synth1m.obj > /dev/null || exit 1; }
for rep in 1 2; do
for t in ${AB_TREES:-head}; do
  if [ $t = head ]; then D=.; else D=ab_$t; fi
  X=""; grep -q no-moving-camera $D/bench.py && X="--no-moving-camera"
  (cd $D && timeout -k 10 300 python bench.py $(eval echo $AB_ARGS) --no-cpu-baseline $X > $GRAFT_REPO_ROOT/gpurun_out/ab_cfg_${t}_$rep.log 2>&1) || exit 1
  python - "$t" "$rep" <<'PY'
import json,sys
l=[x for x in open(f"gpurun_out/ab_cfg_{sys.argv[1]}_{sys.argv[2]}.log") if x.startswith("{")][-1]
d=json.loads(l); print(sys.argv[1], sys.argv[2], d["frame_ms"], d["render_kernel_ms"])
PY
done; done
