# bench.py frame time per library variant (RM_LIB), interleaved A/B/A/B:
# one ms_per_step line per run.  Usage: bash tools/variant_bench_frames.sh OUT lib.so ... (extra bench args in BENCH_ARGS)
set -e
out=$1; shift
for rep in 1 2; do
  for lib in "$@"; do
    RM_LIB=$lib timeout -k 10 120 python bench.py --steps 100 --cpu-seconds 0 $BENCH_ARGS > gpurun_out/vbf.json 2>/dev/null
    python -c "import json,sys;d=json.load(open('gpurun_out/vbf.json'));print('$(basename $lib)',round(d['ms_per_step'],4),round(d['kernel_ms'],4),d['frame_check']['result'])" >> $out
  done
done
