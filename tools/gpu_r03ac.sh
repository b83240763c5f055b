#!/bin/bash
# round 3: the N > 1 bench path rehearsed on one GPU: two ranks over gloo
# (RCCL refuses two ranks on one device), and the 8-shard C4 share
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03ac
mkdir -p $O
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
    bench.py --gpus 2 --steps 10 --warmup 2 --backend gloo --cpu-seconds 0 > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { tail -20 $O/bench_n2_gloo.err; exit 1; }
tail -1 $O/bench_n2_gloo.json | cut -c1-400
timeout -k 10 300 python tools/share_floor.py T 4096 4096 256 16 8 0 P0 > $O/share_floor_C4.json 2> $O/share_floor.err || { tail -5 $O/share_floor.err; exit 1; }
cat $O/share_floor_C4.json
