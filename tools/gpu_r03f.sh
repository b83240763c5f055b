#!/bin/bash
# round 3: tests + bench + PMC of the C3 kernel after the settle exit
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log
[ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" $O/pytest.log | head -60; exit $rc; }
bash tools/pmc_profile.sh T4096r03 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['executed_ray_steps_per_s'], d['ms_per_step'], d['kernel_ms'], d['roofline']['frac'])"
