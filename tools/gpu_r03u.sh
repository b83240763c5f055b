#!/bin/bash
# round 3: backface shadow skip: frames against the build without it (bit
# identity), GPU suite, kernel A/B on every config
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
SCENES=O,OG,T SIZE=512 timeout -k 10 400 python tools/lib_equal.py raymarching_amd/librm.so raymarching_amd/variants/librm_noback.so > $O/lib_equal.jsonl 2> $O/lib_equal.err
rc=$?; cat $O/lib_equal.jsonl; [ $rc -ne 0 ] && { tail -20 $O/lib_equal.err; exit $rc; }
OUTDIR=r03u CONFIGS=C3,C4share,C2P1,O4096,C5frame,C5share LIBS=raymarching_amd/variants/librm_noback.so bash tools/gpu_r03k.sh
