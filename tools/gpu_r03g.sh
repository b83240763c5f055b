#!/bin/bash
# round 3: scene-O soft-shadow settle exit and plane runs: bit-identity of the
# variants (tools/lib_equal.py) and their kernel times on the O configs
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r03g}
mkdir -p $O
V=raymarching_amd/variants
LIBS=${LIBS:-$(ls $V/librm_*.so)}
SCENES=O,OG SIZE=512 timeout -k 10 400 python tools/lib_equal.py $LIBS > $O/lib_equal.jsonl 2> $O/lib_equal.err
rc=$?; cat $O/lib_equal.jsonl; [ $rc -ne 0 ] && { tail -20 $O/lib_equal.err; exit $rc; }
CONFIGS=O4096,C5frame,C5share timeout -k 10 600 python tools/variant_bench.py $LIBS > $O/variants.jsonl 2> $O/variants.err || { tail -20 $O/variants.err; exit 1; }
cat $O/variants.jsonl
