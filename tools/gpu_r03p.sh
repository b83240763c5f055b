#!/bin/bash
# round 3: frames of the default build against the previous defaults (bit
# identity, tools/lib_equal.py), the GPU suite, and the kernel A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r03p}
mkdir -p $O
SCENES=O,OG,T SIZE=512 timeout -k 10 400 python tools/lib_equal.py raymarching_amd/librm.so raymarching_amd/variants/librm_prev.so > $O/lib_equal.jsonl 2> $O/lib_equal.err
rc=$?; cat $O/lib_equal.jsonl; [ $rc -ne 0 ] && { tail -20 $O/lib_equal.err; exit $rc; }
LIBS=raymarching_amd/variants/librm_prev.so bash tools/gpu_r03k.sh
