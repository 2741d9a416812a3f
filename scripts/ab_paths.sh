#!/bin/bash
# A/B of camera-path frame times (scripts/debug_path_state.py) for HEAD and ab_prev/ on one box.
set -u
cd "${GRAFT_REPO_ROOT}"
python -m eray_amd.meshgen --triangles 1000000 --seed 1234 -o /tmp/synth1m.obj > /dev/null || exit 1
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o /tmp/standin70k.obj > /dev/null || exit 1
for t in head prev head prev; do
  if [ $t = head ]; then D=.; else D=ab_prev; fi
  echo "== $t"
  (cd $D && timeout -k 10 200 python scripts/debug_path_state.py /tmp/synth1m.obj 7680 4320 20 2>&1 | grep -E "static|path 2") || exit 1
  (cd $D && timeout -k 10 200 python scripts/debug_path_state.py /tmp/standin70k.obj 1920 1080 40 2>&1 | grep -E "static|path 2") || exit 1
done
