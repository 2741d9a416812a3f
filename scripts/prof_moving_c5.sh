set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out /tmp/eray_meshes
export TMPDIR=/tmp
python -m eray_amd.meshgen --triangles 1000000 --seed 1234 -o /tmp/eray_meshes/synth1m.obj > /dev/null || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mv_c5 -o run --output-format csv -- \
  python scripts/moving_camera.py --mesh /tmp/eray_meshes/synth1m.obj --width 7680 --height 4320 --frames 40 > gpurun_out/prof_mv_c5.log 2>&1
echo rc=$?; tail -1 gpurun_out/prof_mv_c5.log
