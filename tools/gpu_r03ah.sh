#!/bin/bash
# round 3: frame interval with and without bench's per-frame timing events
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03ah
mkdir -p $O
: > $O/events.jsonl
for rep in 1 2; do
  for ne in 0 1; do
    RM_BENCH_NO_EVENTS=$ne timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 40 > $O/b.json 2> $O/b.err || { tail -3 $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); print(json.dumps(dict(rep=$rep, no_events=$ne, ms_per_step=d['ms_per_step'], kernel_ms=d['kernel_ms'])))" >> $O/events.jsonl
  done
done
cat $O/events.jsonl
