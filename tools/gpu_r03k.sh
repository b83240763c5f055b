#!/bin/bash
# round 3: GPU test suite, then kernel A/B of the default build against
# variants (LIBS) on the scene-O configs (CONFIGS)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r03k}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" $O/pytest.log | head -80; exit $rc; }
CONFIGS=${CONFIGS:-O4096,C5frame,C5share} timeout -k 10 600 python tools/variant_bench.py raymarching_amd/librm.so ${LIBS:-} > $O/variants.jsonl 2> $O/variants.err || { tail -20 $O/variants.err; exit 1; }
python - <<PY
import json
for l in open("$O/variants.jsonl"):
    d = json.loads(l)
    if d["schedule"] == 1: print(d["lib"], d["config"], round(d["kernel_ms"], 4))
PY
