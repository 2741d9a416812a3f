#!/bin/bash
# Camera-path tests (both modes), then an A/B on one box: moving-camera loops over binned meshes
# enqueued directly (the default since this A/B) or replayed from captured graphs
# (ERAY_MULTI_GRAPHS=1; the A/B was run with the opposite default, ERAY_MULTI_DIRECT=1 selecting
# the direct form).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ab_multi
mkdir -p $OUT /tmp/eray_meshes
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_camera_path.py tests/test_gpu_ring.py > $OUT/tests.log 2>&1
rc=$?; tail -2 $OUT/tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAIL\|Error" $OUT/tests.log | head -60; exit $rc; }
ERAY_MULTI_GRAPHS=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_camera_path.py tests/test_gpu_ring.py > $OUT/tests_direct.log 2>&1
rc=$?; tail -2 $OUT/tests_direct.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAIL\|Error" $OUT/tests_direct.log | head -60; exit $rc; }
python -m eray_amd.meshgen --triangles 1000000 --seed 1234 -o /tmp/eray_meshes/synth1m.obj > /dev/null || exit 1
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o /tmp/eray_meshes/standin70k.obj > /dev/null || exit 1
for rep in 1 2; do
  for mode in direct graphs; do
    if [ $mode = graphs ]; then export ERAY_MULTI_GRAPHS=1; else unset ERAY_MULTI_GRAPHS; fi
    for cfg in "c5:/tmp/eray_meshes/synth1m.obj 7680 4320 24" "n1:/tmp/eray_meshes/standin70k.obj 3840 2160 64" "c3:/tmp/eray_meshes/standin70k.obj 1920 1080 100"; do
      name=${cfg%%:*}; set -- ${cfg#*:}
      timeout -k 10 200 python scripts/moving_camera.py --mesh $1 --width $2 --height $3 --frames $4 > $OUT/${mode}${rep}_$name.log 2>&1 || { tail -5 $OUT/${mode}${rep}_$name.log; exit 1; }
      echo "$mode$rep $name $(grep moving $OUT/${mode}${rep}_$name.log)"
    done
  done
done
