#!/bin/bash
# round 3: scene-O variants (settle test as one minimum, 7 waves, thickness
# loop unrolled by 2) on the O configs, then the dispatch order under motion
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
V=raymarching_amd/variants
CONFIGS=O4096,C5frame,C5share timeout -k 10 600 python tools/variant_bench.py raymarching_amd/librm.so $V/librm_smin.so $V/librm_w7.so $V/librm_th2.so > $O/variants.jsonl 2> $O/variants.err || { tail -20 $O/variants.err; exit 1; }
python - <<PY
import json
for l in open("$O/variants.jsonl"):
    d = json.loads(l)
    if d["schedule"] == 1: print(d["lib"], d["config"], round(d["kernel_ms"], 4))
PY
bash tools/gpu_r03n.sh
