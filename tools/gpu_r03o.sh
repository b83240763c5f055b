#!/bin/bash
# round 3: GPU suite + kernel A/B (tools/gpu_r03k.sh), then the C3 bench line
# with its post passes (FXAA, bloom)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_r03k.sh || exit 1
O=gpurun_out/${OUTDIR:-r03k}
timeout -k 10 300 python bench.py --cpu-seconds 0 > $O/bench_C3.json 2> $O/bench_C3.err || { tail -5 $O/bench_C3.err; exit 1; }
python -c "
import json; d=json.load(open('$O/bench_C3.json'))
print('C3', d['value'], d['ms_per_step'], d['kernel_ms'], 'fxaa', d['post_pass']['ms'], 'bloom', d['bloom_pass']['ms'])"
