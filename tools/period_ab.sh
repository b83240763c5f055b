#!/bin/bash
# bench C3 frame time and kernel time for dispatch-order sort periods (RM_SCHED_PERIOD)
cd "${GRAFT_REPO_ROOT:-.}"
for p in ${PERIODS:-1 2 4 8 1 4}; do
  RM_SCHED_PERIOD=$p timeout -k 10 200 python bench.py --cpu-seconds 0 --steps 300 ${BENCH_ARGS:-} > gpurun_out/period_$p.json 2>/dev/null || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print('period', sys.argv[2], 'ms/step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4), 'gap_us', round(1000*(d['ms_per_step']-d['kernel_ms']),1))" gpurun_out/period_$p.json $p
done
