#!/bin/bash
# round 3: scene O with the rolled AO loop: GPU suite, PMC (HBM bytes), C5 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03aa
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" $O/pytest.log | head -60; exit $rc; }
bash tools/pmc_profile.sh O8192r03c --scene O --size 8192 --max-steps 512 || exit 1
timeout -k 10 300 python bench.py --scene O --size 8192 --max-steps 512 --steps 10 > $O/bench_C5.json 2> $O/bench_C5.err || { tail -5 $O/bench_C5.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_C5.json')); print('C5', d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'], d['roofline']['traffic'])"
