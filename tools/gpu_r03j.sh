#!/bin/bash
# round 3: full GPU test suite on the default build
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" $O/pytest.log | head -80; exit $rc; }
timeout -k 10 300 python bench.py --scene O --size 8192 --max-steps 512 --steps 10 --cpu-seconds 0 > $O/bench_C5.json 2> $O/bench_C5.err || { tail -5 $O/bench_C5.err; exit 1; }
timeout -k 10 300 python bench.py --cpu-seconds 0 > $O/bench_C3.json 2> $O/bench_C3.err || { tail -5 $O/bench_C3.err; exit 1; }
python -c "
import json
for f in ('bench_C5','bench_C3'):
    d=json.load(open('$O/'+f+'.json')); print(f, d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])"
