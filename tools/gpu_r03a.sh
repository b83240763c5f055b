#!/bin/bash
# round 3, first GPU pass: scene-O compact code (bit identity, A/B, I-cache PMC)
# and the full-size step-map parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03a
mkdir -p $O
BASE=raymarching_amd/variants/librm_o_base.so
timeout -k 10 400 python tools/lib_equal.py $BASE raymarching_amd/librm.so > $O/equal.json 2> $O/equal.err || { echo "equal failed"; cat $O/equal.json; tail -5 $O/equal.err; exit 1; }
cat $O/equal.json
CONFIGS=O4096,C5frame timeout -k 10 400 python tools/variant_bench.py $BASE raymarching_amd/librm.so > $O/ab.jsonl 2> $O/ab.err || { echo "ab failed"; tail -5 $O/ab.err; exit 1; }
cat $O/ab.jsonl
for v in base compact; do
  lib=$BASE; [ $v = compact ] && lib=raymarching_amd/librm.so
  RM_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $O/pmc_$v -o run -- python bench.py --scene O --size 4096 --max-steps 512 --steps 5 --warmup 2 --cpu-seconds 0 > $O/pmc_$v.log 2>&1 || { echo "pmc $v failed"; tail -5 $O/pmc_$v.log; exit 1; }
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -5 $O/pytest.log
exit $rc
