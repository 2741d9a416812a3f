#!/bin/bash
# Round 4: C5's frame on one GPU and one rank's share of the 8-GPU split (rank 3: row0 = 12,
# bands of 4 rows every 32), each timed per dispatch (c5_probe.py), under rocprofv3's kernel trace,
# and through counter passes (each counter group its own run) for their traffic and wait fraction.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04r}
mkdir -p $OUT
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for w in full:"--shares= --shapes default --no-empty --launches 20" share3:"--no-full --shares 3 --shapes default --no-empty --launches 40"; do
  name=${w%%:*}; args=${w#*:}
  timeout -k 10 300 python scripts/c5_probe.py $args > $OUT/$name.json 2> $OUT/$name.err || { tail -20 $OUT/$name.err; exit 1; }
  cat $OUT/$name.json
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$OUT/prof_$name -o run -- python3 $R/scripts/c5_probe.py $args > $R/$OUT/prof_$name.log 2>&1) || { tail -20 $OUT/prof_$name.log; exit 1; }
  mkdir -p $OUT/pmc_$name
  for g in "sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "fetch FETCH_SIZE" "write WRITE_SIZE GRBM_GUI_ACTIVE"; do
    set -- $g; gname=$1; shift
    (cd /tmp && timeout -k 10 150 rocprofv3 --pmc "$@" --kernel-include-regex 'frame_kernel|fill_kernel' --output-format csv -d $R/$OUT/pmc_$name/$gname -o $gname -- python3 $R/scripts/c5_probe.py $args > $R/$OUT/pmc_$name/$gname.log 2>&1)
    rc=$?; echo "pmc $name/$gname rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/pmc_$name/$gname.log; exit $rc; }
  done
done
# main.rs's graph at the hit texel (no texture reads) against the textures, same box
timeout -k 10 300 python scripts/ab_probe.py --configs ns1,ns1ex,ns4,ns4ex,c2,c2ex > $OUT/material_ab.json 2> $OUT/material_ab.err || { tail -20 $OUT/material_ab.err; exit 1; }
cat $OUT/material_ab.json
# cameras per multi-camera build: 16 (product) against 32 / 64 at 70k faces (k64: 8 at 1M)
TAG=${TAG:-r04r}/kcam LIBS="product k32 k64" ROUNDS=2 CONFIGS=moving_ns,moving_c5 bash scripts/ab_session.sh
