#!/bin/bash
# SQ counters of the static C3 frame kernel for HEAD and a build of an earlier commit in ab_<name>/.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/abpmc /tmp/eray_meshes
export TMPDIR=/tmp
M=/tmp/eray_meshes
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o $M/standin70k.obj > /dev/null || exit 1
for t in head ${AB_TREE:-r01}; do
  if [ $t = head ]; then D=.; else D=ab_$t; fi
  X=""; grep -q no-moving-camera $D/bench.py && X="--no-moving-camera"
  (cd $D && timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY \
      --kernel-include-regex 'frame_kernel' --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/abpmc/$t -o run -- \
      python bench.py --mesh $M/standin70k.obj --steps 50 --warmup 5 --no-cpu-baseline $X > $GRAFT_REPO_ROOT/gpurun_out/abpmc/$t.log 2>&1) || exit 1
  echo "$t done"
done
