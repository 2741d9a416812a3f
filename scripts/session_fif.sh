set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out /tmp/eray_meshes
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o /tmp/eray_meshes/standin70k.obj > /dev/null || exit 1
timeout -k 10 400 python -u scripts/frames_in_flight.py --big > gpurun_out/fif.log 2>&1; rc=$?
cat gpurun_out/fif.log | grep -v amdgpu.ids
exit $rc
