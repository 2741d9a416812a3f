#!/bin/bash
# Round-3 session f: detail share A/B with the spill-free dense build, its trace, frames in flight at 4K/70k.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out /tmp/eray_meshes
export TMPDIR=/tmp
M=/tmp/eray_meshes
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o $M/standin70k.obj > /dev/null || exit 1
: > gpurun_out/ab_share.log
for rep in 1 2; do
  for v in base w3s25 w3s17 w3s3; do
    if [ $v = base ]; then L=eray_amd/lib/liberay_hip.so; else L=eray_amd/lib/liberay_hip_$v.so; fi
    out=$(ERAY_LIB=$L timeout -k 10 120 python scripts/ab_flags.py $M/standin70k.obj 3840 2160 0 2>/dev/null | tail -1)
    rc=$?
    echo "$v $out" | tee -a gpurun_out/ab_share.log
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
timeout -k 10 120 env ERAY_LIB=eray_amd/lib/liberay_hip_trace.so python scripts/wg_trace.py $M/standin70k.obj 3840 2160 > gpurun_out/trace_4k70k_b1.log 2>&1 || exit $?
grep -v amdgpu gpurun_out/trace_4k70k_b1.log | head -8
timeout -k 10 200 python - > gpurun_out/fif_4k.log 2>&1 <<'PY' || exit $?
import sys; sys.argv = ["x"]
sys.path.insert(0, ".")
import torch
from scripts.frames_in_flight import run
from eray_amd import capi
from eray_amd.objfile import load_obj_file
ctx = capi.Context(0)
st = torch.cuda.Stream(); ctx.set_stream(st.cuda_stream); torch.cuda.set_stream(st)
big = load_obj_file("/tmp/eray_meshes/standin70k.obj")
run(ctx, "70k 3840x2160", big, 3840, 2160, 64, per_launch=((1, 1), (2, 2)))
run(ctx, "C3", big, 1920, 1080, 128, per_launch=((1, 1), (2, 2), (4, 4)))
PY
grep -v amdgpu gpurun_out/fif_4k.log
