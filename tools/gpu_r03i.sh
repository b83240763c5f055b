#!/bin/bash
# round 3: settle-test period (scene O every 8/16/32 steps, scene T every 1/2/4)
# and scene-O phase ablations (SSS, soft shadow) on the C5 frame
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
V=raymarching_amd/variants
L="raymarching_amd/librm.so $V/librm_o16.so $V/librm_o32.so $V/librm_t2.so $V/librm_t4.so"
SCENES=O,OG,T SIZE=512 timeout -k 10 400 python tools/lib_equal.py $L > $O/lib_equal.jsonl 2> $O/lib_equal.err
rc=$?; cat $O/lib_equal.jsonl; [ $rc -ne 0 ] && { tail -20 $O/lib_equal.err; exit $rc; }
timeout -k 10 600 python tools/variant_bench.py $L > $O/variants.jsonl 2> $O/variants.err || { tail -20 $O/variants.err; exit 1; }
CONFIGS=C5frame timeout -k 10 300 python tools/variant_bench.py $V/librm_abl_sss.so $V/librm_abl_sha.so >> $O/variants.jsonl 2>> $O/variants.err || { tail -20 $O/variants.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/r03i/variants.jsonl"):
    d = json.loads(l)
    if d["schedule"] == 1: print(d["lib"], d["config"], round(d["kernel_ms"], 4))
PY
