# bench.py C3 frame time under environment knobs, interleaved twice:
# one line per run.  Usage: bash tools/knob_ab.sh OUT 'ENV=..' 'ENV=..' ...
set -e
out=$1; shift
for rep in 1 2; do
  for kv in "$@"; do
    env $kv timeout -k 10 120 python bench.py --steps 100 --cpu-seconds 0 $BENCH_ARGS > gpurun_out/knob.json 2>/dev/null
    python -c "import json;d=json.load(open('gpurun_out/knob.json'));print('$kv',round(d['ms_per_step'],4),round(d['kernel_ms'],4),d['frame_check']['result'])" >> $out
  done
done
