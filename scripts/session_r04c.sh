#!/bin/bash
# Round 4 diagnostics: 3840x2160 / 70k bin statistics and workgroup timelines (trace build), C5's
# frame and band shares per launch shape, the fill microbenchmark per dispatch.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04c}
mkdir -p $OUT /tmp/eray_meshes
export TMPDIR=/tmp
M=/tmp/eray_meshes
timeout -k 10 120 python -m eray_amd.meshgen --triangles 69451 --seed 42 -o $M/standin70k.obj > /dev/null || exit 1
timeout -k 10 120 python scripts/bin_stats.py $M/standin70k.obj 3840 2160 > $OUT/bin_stats_ns.txt 2>&1 || { cat $OUT/bin_stats_ns.txt; exit 1; }
ERAY_LIB=eray_amd/lib/liberay_hip_trace.so timeout -k 10 120 python scripts/wg_trace.py $M/standin70k.obj 3840 2160 > $OUT/trace_ns.txt 2>&1 || { tail -20 $OUT/trace_ns.txt; exit 1; }
ERAY_LIB=eray_amd/lib/liberay_hip_trace.so timeout -k 10 120 python scripts/wg_trace.py objects/cube.obj 1920 1080 > $OUT/trace_c2.txt 2>&1 || { tail -20 $OUT/trace_c2.txt; exit 1; }
timeout -k 10 300 python scripts/c5_probe.py > $OUT/c5_probe.json 2> $OUT/c5_probe.err || { tail -20 $OUT/c5_probe.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/fill_mlp -o fill -- scripts/microbench/fill_mlp > $OUT/fill_mlp.txt 2>&1 || { tail -20 $OUT/fill_mlp.txt; exit 1; }
