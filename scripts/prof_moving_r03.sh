#!/bin/bash
# Kernel traces of the moving-camera loop (scripts/moving_camera.py) at C5's frame (1M faces,
# 7680x4320) and 3840x2160 / 70k: per-kernel statistics and the last kernels' timeline.
set -u
cd "${GRAFT_REPO_ROOT}"
OUT=gpurun_out/${TAG:-mv}
mkdir -p $OUT /tmp/eray_meshes
export TMPDIR=/tmp
python -m eray_amd.meshgen --triangles 1000000 --seed 1234 -o /tmp/eray_meshes/synth1m.obj > /dev/null || exit 1
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o /tmp/eray_meshes/standin70k.obj > /dev/null || exit 1
for cfg in "c5:/tmp/eray_meshes/synth1m.obj 7680 4320 24" "n1:/tmp/eray_meshes/standin70k.obj 3840 2160 64"; do
  name=${cfg%%:*}; set -- ${cfg#*:}
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/prof_$name -o run --output-format csv -- \
    python scripts/moving_camera.py --mesh $1 --width $2 --height $3 --frames $4 > $OUT/$name.log 2>&1 || { tail -5 $OUT/$name.log; exit 1; }
  tail -1 $OUT/$name.log
  f=$(ls $OUT/prof_$name/*/run_kernel_trace.csv 2>/dev/null || ls $OUT/prof_$name/run_kernel_trace.csv)
  python scripts/timeline.py $f 120 > $OUT/${name}_timeline.txt
done
