#!/bin/bash
# round 3: pytest -m gpu (full-size step maps, multi-rank C ABI through the
# RCCL stand-in, C++ adapter RGBA8), bench under motion, headless C++ frame rate
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -4 $O/pytest.log
[ $rc -ne 0 ] && exit $rc
for v in "static:" "walk:--walk" "walk_rowmajor:--walk --schedule rowmajor" "static_rowmajor:--schedule rowmajor"; do
  name=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python bench.py --cpu-seconds 0 $a > $O/bench_$name.json 2> $O/bench_$name.err || { echo "bench $name failed"; tail -3 $O/bench_$name.err; exit 1; }
  RM_LAT_TILES=0 timeout -k 10 300 python bench.py --cpu-seconds 0 $a > $O/bench_${name}_nolat.json 2> $O/bench_${name}_nolat.err || { echo "bench $name nolat failed"; exit 1; }
done
for f in $O/bench_*.json; do python -c "import json,sys; d=json.load(open('$f')); print('$f', round(d['value']/1e12,4), 'Tsteps/s', round(d['ms_per_step'],4), 'ms', round(d['kernel_ms'],4))"; done
timeout -k 10 300 apps/raymarch_headless --scene template.frag --w 4096 --h 4096 --steps 256 --time-freeze --frames 200 --warmup 50 > $O/headless_C3.json 2> $O/headless_C3.err || { echo "headless failed"; cat $O/headless_C3.err; exit 1; }
cat $O/headless_C3.json
timeout -k 10 300 apps/raymarch_headless --scene template.frag --w 4096 --h 4096 --steps 256 --time-freeze --frames 200 --warmup 50 --stats > $O/headless_C3_stats.json 2>&1
cat $O/headless_C3_stats.json
