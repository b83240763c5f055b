#!/bin/bash
# round 3: scene-T soft-shadow settle exit: bit identity, A/B, tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
BASE=raymarching_amd/variants/librm_t_nosettle.so
SCENES=T,S0 timeout -k 10 400 python tools/lib_equal.py $BASE raymarching_amd/librm.so > $O/equal.json 2> $O/equal.err; rc=$?
cat $O/equal.json; [ $rc -ne 0 ] && { tail -5 $O/equal.err; exit 1; }
SCENES=T SIZE=4096 timeout -k 10 400 python tools/lib_equal.py $BASE raymarching_amd/librm.so > $O/equal4096.json 2>> $O/equal.err || { cat $O/equal4096.json; exit 1; }
cat $O/equal4096.json
CONFIGS=C3,C4share,C2P1 timeout -k 10 400 python tools/variant_bench.py $BASE raymarching_amd/librm.so > $O/ab.jsonl 2> $O/ab.err || { tail -5 $O/ab.err; exit 1; }
cat $O/ab.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python bench.py --cpu-seconds 0 > $O/bench.json 2> $O/bench.err && python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['kernel_ms'])"
