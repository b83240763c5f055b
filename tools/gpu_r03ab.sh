#!/bin/bash
# round 3: backface shadow skip in scene plugins: GPU suite, plugin frame times
# against the build without it
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03ab
mkdir -p $O
[ -n "${NOTEST:-}" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
[ -n "${NOTEST:-}" ] || tail -2 $O/pytest.log
[ -z "${NOTEST:-}" ] && [ $rc -ne 0 ] && { grep -B5 -A30 "FAILED\|Error" $O/pytest.log | head -60; exit $rc; }
: > $O/plugin_bench.jsonl
for lib in ${PLIBS:-raymarching_amd/librm.so raymarching_amd/variants/librm_prevplug.so}; do
  RM_LIB=$(pwd)/$lib timeout -k 10 300 python tools/plugin_bench.py > $O/pb.jsonl 2> $O/pb.err || { tail -5 $O/pb.err; exit 1; }
  python -c "
import json
for l in open('$O/pb.jsonl'):
    d = json.loads(l); d['lib'] = '$lib'; print(json.dumps(d))" >> $O/plugin_bench.jsonl
done
cat $O/plugin_bench.jsonl
