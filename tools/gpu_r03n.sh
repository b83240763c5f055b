#!/bin/bash
# round 3: dispatch order under motion after the settle exits: bench --walk
# and the still pose, adaptive order with sort-key dilation 0/2/4 and row-major,
# two repeats each (40 timed frames)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
: > $O/sched_walk.jsonl
for rep in 1 2; do
  for cfg in "adaptive 0" "adaptive 2" "adaptive 4" "rowmajor 0"; do
    set -- $cfg
    for mode in walk static; do
      a=""; [ $mode = walk ] && a="--walk"
      RM_SCHED_DILATE=$2 timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 40 --schedule $1 $a ${BENCH_ARGS:-} > $O/b.json 2> $O/b.err || { echo "bench failed $cfg $mode"; tail -3 $O/b.err; exit 1; }
      python -c "import json; d=json.load(open('$O/b.json')); print(json.dumps(dict(rep=$rep, mode='$mode', schedule='$1', dilate=$2, value=d['value'], ms_per_step=d['ms_per_step'], kernel_ms=d['kernel_ms'], frame_stream_ms=d['frame_stream_ms'])))" >> $O/sched_walk.jsonl
    done
  done
done
python - <<PY
import json, collections
r = collections.defaultdict(list)
for l in open("$O/sched_walk.jsonl"):
    d = json.loads(l); r[(d["mode"], d["schedule"], d["dilate"])].append(d["ms_per_step"])
for k, v in sorted(r.items()): print(k, [round(x, 4) for x in v])
PY
