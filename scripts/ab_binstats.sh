set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p /tmp/eray_meshes gpurun_out
M=/tmp/eray_meshes
python -m eray_amd.meshgen --triangles 69451 --seed 42 -o $M/standin70k.obj > /dev/null || exit 1
timeout -k 10 120 python scripts/bin_stats.py $M/standin70k.obj 1920 1080 > gpurun_out/bs_head.log 2>&1; echo head $?; tail -1 gpurun_out/bs_head.log
cd ab_r01 && timeout -k 10 120 python ../scripts/bin_stats.py $M/standin70k.obj 1920 1080 > ../gpurun_out/bs_r01.log 2>&1; echo r01 $?; tail -1 ../gpurun_out/bs_r01.log
