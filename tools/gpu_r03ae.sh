#!/bin/bash
# round 3: dispatch-order sort period 4 vs 8 after the skips, still and walking
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03ae
mkdir -p $O
: > $O/period.jsonl
for rep in 1 2; do
  for pd in ${PERIODS:-4 8 2}; do
    for mode in static walk; do
      a=""; [ $mode = walk ] && a="--walk"
      RM_SCHED_PERIOD=$pd timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 40 $a > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
      python -c "import json; d=json.load(open('$O/b.json')); print(json.dumps(dict(rep=$rep, period=$pd, mode='$mode', value=d['value'], ms_per_step=d['ms_per_step'], kernel_ms=d['kernel_ms'])))" >> $O/period.jsonl
    done
  done
done
python - <<PY
import json, collections
r = collections.defaultdict(list)
for l in open("$O/period.jsonl"):
    d = json.loads(l); r[(d["mode"], d["period"])].append(round(d["ms_per_step"], 4))
for k, v in sorted(r.items()): print(k, v)
PY
