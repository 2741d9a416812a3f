#!/bin/bash
# Camera paths with frames in flight over binned meshes: path + ring tests, then the C3 and 4K/70k bench lines (moving camera).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r03k}
mkdir -p $OUT /tmp/eray_meshes
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_camera_path.py tests/test_gpu_ring.py > $OUT/tests.log 2>&1
rc=$?; tail -5 $OUT/tests.log; [ $rc -eq 0 ] || { grep -B5 -A30 "FAIL\|Error" $OUT/tests.log | head -80; exit $rc; }
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o /tmp/eray_meshes/standin70k.obj > /dev/null || exit 1
for cfg in "c3:--mesh /tmp/eray_meshes/standin70k.obj --steps 100" "n1:--mesh /tmp/eray_meshes/standin70k.obj --width 3840 --height 2160 --steps 50"; do
  name=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 300 python bench.py $args --no-cpu-baseline > $OUT/$name.log 2>&1 || exit $?
  grep '^{' $OUT/$name.log | tail -1 > $OUT/$name.json
  python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['ms_per_step'], 'moving', d['moving_camera']['device_ms_per_frame'], 'aa', (d.get('anti_aliased') or {}).get('frame_ms'))"
done
