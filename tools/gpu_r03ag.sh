#!/bin/bash
# round 3: workgroup tiling after the skips: 8x8 one-wave tiles (default) vs
# 16x4 one-wave tiles vs 16x16 four-wave workgroups, every config
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03ag
mkdir -p $O
: > $O/tiling.jsonl
for k in tile8 tile16x4 tile16; do
  RM_KERNEL=$k timeout -k 10 400 python tools/variant_bench.py raymarching_amd/librm.so > $O/v.jsonl 2> $O/v.err || { tail -5 $O/v.err; exit 1; }
  cat $O/v.jsonl >> $O/tiling.jsonl
done
python - <<PY
import json
for l in open("$O/tiling.jsonl"):
    d = json.loads(l)
    if d["schedule"] == 1: print(d["kernel"], d["config"], round(d["kernel_ms"], 4))
PY
