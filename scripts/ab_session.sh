#!/bin/bash
# Same-box A/B: scripts/ab_probe.py with each library of $LIBS (names under eray_amd/lib/,
# liberay_hip_<name>.so; "product" = liberay_hip.so), alternating, $ROUNDS times.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab}
mkdir -p $OUT
export TMPDIR=/tmp
for r in $(seq 1 ${ROUNDS:-2}); do
  for l in ${LIBS:-base product}; do
    lib=eray_amd/lib/liberay_hip_$l.so
    [ $l = product ] && lib=eray_amd/lib/liberay_hip.so
    ERAY_LIB=$PWD/$lib timeout -k 10 300 python scripts/ab_probe.py --configs ${CONFIGS:-c2,c3,ns1,ns4} >> $OUT/ab.jsonl 2>> $OUT/ab.err || { tail -20 $OUT/ab.err; exit 1; }
  done
done
python - $OUT/ab.jsonl <<'PY'
import json, sys, collections
rows = [json.loads(l) for l in open(sys.argv[1])]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    for k, v in r.items():
        if k != "lib":
            agg[k][r["lib"]].append(v.get("launch_span_ms", v.get("device_ms_per_frame", v.get("frame_ms"))) * 1e3)
for k, d in agg.items():
    print(k, {l: [round(x, 2) for x in v] for l, v in d.items()})
PY
