#!/bin/bash
# round 3: latency tiles after the backface skip: count sweep (RM_LAT_TILES)
# and the settle exit inside them (RM_LAT_SETTLE), on the T configs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
: > $O/lat.jsonl
for n in 0 512 2048 8192; do
  RM_LAT_TILES=$n CONFIGS=C3,C4share,C2P1 timeout -k 10 300 python tools/variant_bench.py raymarching_amd/librm.so raymarching_amd/variants/librm_latsettle.so > $O/v.jsonl 2> $O/v.err || { tail -5 $O/v.err; exit 1; }
  python -c "
import json
for l in open('$O/v.jsonl'):
    d = json.loads(l); d['lat_tiles'] = $n; print(json.dumps(d))" >> $O/lat.jsonl
done
python - <<PY
import json
for l in open("$O/lat.jsonl"):
    d = json.loads(l)
    if d["schedule"] == 1: print(d["lat_tiles"], d["lib"], d["config"], round(d["kernel_ms"], 4))
PY
