#!/bin/bash
# round 3: rolled AO / normal probe loops (fewer live registers, fewer scene-O
# spills): bit identity and kernel A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O
V=raymarching_amd/variants
SCENES=O,OG,T SIZE=512 timeout -k 10 400 python tools/lib_equal.py raymarching_amd/librm.so $V/librm_aorolled.so $V/librm_nrolled.so $V/librm_bothrolled.so > $O/lib_equal.jsonl 2> $O/lib_equal.err
rc=$?; cat $O/lib_equal.jsonl; [ $rc -ne 0 ] && { tail -20 $O/lib_equal.err; exit $rc; }
timeout -k 10 600 python tools/variant_bench.py raymarching_amd/librm.so $V/librm_aorolled.so $V/librm_nrolled.so $V/librm_bothrolled.so > $O/variants.jsonl 2> $O/variants.err || { tail -20 $O/variants.err; exit 1; }
python - <<PY
import json
for l in open("$O/variants.jsonl"):
    d = json.loads(l)
    if d["schedule"] == 1: print(d["lib"], d["config"], round(d["kernel_ms"], 4))
PY
