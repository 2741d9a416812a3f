set -u
mkdir -p gpurun_out/aa
for v in ${VARIANTS:-"" nosearch noshade}; do
  lib=eray_amd/lib/liberay_hip${v:+_$v}.so
  echo "== $v"
  ERAY_LIB=$PWD/$lib timeout -k 10 120 python scripts/aa_probe.py 2>&1 | grep -v amdgpu | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['frame_ms'])" || exit 1
done
