#!/bin/bash
# One GPU session for A/B work: variant timing (tools/variant_bench.py) of the
# libraries given in LIBS over CONFIGS, then optional bench.py runs (BENCH_ARGS_1..3).
# Output -> gpurun_out/<TAG>_*.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-ab}
if [ -n "${LIBS:-}" ]; then
  timeout -k 10 ${VB_TIMEOUT:-400} python tools/variant_bench.py $LIBS > gpurun_out/${TAG}_variants.jsonl 2> gpurun_out/${TAG}_variants.err || { echo "variant bench failed"; tail -5 gpurun_out/${TAG}_variants.err; exit 3; }
  cat gpurun_out/${TAG}_variants.jsonl
fi
for k in 1 2 3; do
  v=BENCH_ARGS_$k
  [ -z "${!v:-}" ] && continue
  timeout -k 10 300 python bench.py --cpu-seconds 0 ${!v} > gpurun_out/${TAG}_bench$k.json 2> gpurun_out/${TAG}_bench$k.err || { echo "bench $k failed"; tail -5 gpurun_out/${TAG}_bench$k.err; exit 4; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['config']['workload'][:40], 'ms/step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4), 'value', '%.4g' % d['value'])" gpurun_out/${TAG}_bench$k.json "${!v}"
done
