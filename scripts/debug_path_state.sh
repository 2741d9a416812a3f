set -u
cd "${GRAFT_REPO_ROOT}"
python -m eray_amd.meshgen --triangles 1000000 --seed 1234 -o /tmp/synth1m.obj > /dev/null || exit 1
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o /tmp/standin70k.obj > /dev/null || exit 1
timeout -k 10 200 python scripts/debug_path_state.py /tmp/synth1m.obj 7680 4320 20 2>&1 | grep -v amdgpu.ids
timeout -k 10 200 python scripts/debug_path_state.py /tmp/standin70k.obj 1920 1080 40 2>&1 | grep -v amdgpu.ids
