#!/bin/bash
# round 3: bench lines after the timing-event change (C3 twice, walking, C5)
# and the kernel trace of the default bench command
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${OUTDIR:-r03ai}
mkdir -p $O
timeout -k 10 300 python bench.py > $O/bench_C3.json 2> $O/bench_C3.err || { tail -5 $O/bench_C3.err; exit 1; }
timeout -k 10 300 python bench.py --cpu-seconds 0 > $O/bench_C3b.json 2> $O/bench_C3b.err || { tail -5 $O/bench_C3b.err; exit 1; }
timeout -k 10 300 python bench.py --walk --cpu-seconds 0 > $O/bench_C3_walk.json 2> $O/bench_C3_walk.err || { tail -5 $O/bench_C3_walk.err; exit 1; }
timeout -k 10 300 python bench.py --scene O --size 8192 --max-steps 512 --steps 10 > $O/bench_C5.json 2> $O/bench_C5.err || { tail -5 $O/bench_C5.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python bench.py --cpu-seconds 0 --steps 20 > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
find $O/trace -name "*kernel_stats.csv" -exec cp {} $O/bench_C3_kernel_stats.csv \;
python - <<PY
import json
for f in ("bench_C3", "bench_C3b", "bench_C3_walk", "bench_C5"):
    d = json.load(open("$O/" + f + ".json"))
    print(f, "%.4g" % d["value"], "ms/step %.4f" % d["ms_per_step"], "kernel %.4f" % d["kernel_ms"], "stream %.4f" % d["frame_stream_ms"], "frac %.3f" % d["roofline"]["frac"])
PY
head -3 $O/bench_C3_kernel_stats.csv | cut -c1-160
