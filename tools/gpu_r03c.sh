#!/bin/bash
# round 3: adaptive order under motion (sort period x key dilation), C4 share floor
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
: > $O/sched_walk.jsonl
for pd in "4 0" "1 0" "2 0" "4 1" "4 2" "1 1" "1 2" "4 4"; do
  set -- $pd
  for mode in walk static; do
    a=""; [ $mode = walk ] && a="--walk"
    RM_SCHED_PERIOD=$1 RM_SCHED_DILATE=$2 timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 40 $a > $O/b.json 2> $O/b.err || { echo "bench failed $pd $mode"; tail -3 $O/b.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b.json')); print(json.dumps(dict(mode='$mode', period=$1, dilate=$2, value=d['value'], ms_per_step=d['ms_per_step'], kernel_ms=d['kernel_ms'], frame_stream_ms=d['frame_stream_ms'])))" >> $O/sched_walk.jsonl
  done
done
for mode in walk static; do
  a=""; [ $mode = walk ] && a="--walk"
  timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 40 --schedule rowmajor $a > $O/b.json 2> $O/b.err || exit 1
  python -c "import json; d=json.load(open('$O/b.json')); print(json.dumps(dict(mode='$mode', schedule='rowmajor', value=d['value'], ms_per_step=d['ms_per_step'], kernel_ms=d['kernel_ms'], frame_stream_ms=d['frame_stream_ms'])))" >> $O/sched_walk.jsonl
done
cat $O/sched_walk.jsonl
timeout -k 10 300 python tools/share_floor.py T 4096 4096 256 16 8 0 P0 > $O/share_floor_C4.json 2> $O/share_floor.err || { tail -5 $O/share_floor.err; exit 1; }
timeout -k 10 300 python tools/share_floor.py T 1920 1080 128 1080 1 0 P1 > $O/share_floor_C2P1.json 2>> $O/share_floor.err || exit 1
cat $O/share_floor_C4.json $O/share_floor_C2P1.json
