#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
BASE=raymarching_amd/variants/librm_t_nosettle.so
SCENES=T SIZE=1024 timeout -k 10 400 python tools/lib_equal.py $BASE raymarching_amd/librm.so > $O/equal.json 2> $O/equal.err; rc=$?
cat $O/equal.json; [ $rc -ne 0 ] && { tail -5 $O/equal.err; exit 1; }
CONFIGS=C3,C4share,C2P1 timeout -k 10 400 python tools/variant_bench.py $BASE raymarching_amd/librm.so > $O/ab.jsonl 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
cat $O/ab.jsonl
for d in 0 2; do RM_SCHED_DILATE=$d CONFIGS=C3,C4share,C2P1 timeout -k 10 400 python tools/variant_bench.py raymarching_amd/librm.so > $O/ab_dilate$d.jsonl 2>> $O/ab.err || exit 1; cat $O/ab_dilate$d.jsonl; done
