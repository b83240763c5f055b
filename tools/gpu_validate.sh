#!/bin/bash
# Round validation on one GPU box: pytest -m gpu (parity figures to
# gpurun_out/parity_TAG.jsonl), smoke(), the C3 bench line and its rocprofv3
# kernel trace, the C5 frame bench, the two-rank gloo rehearsal (C3), and with
# PMC=1 the PMC passes of C3 / C5 (tools/pmc_profile.sh) and of FXAA / bloom
# (tools/pmc_post.sh).  Every GPU step has its own time limit; the first
# failure ends the script.  Usage: [PMC=1] [SKIP_TESTS=1] tools/gpu_validate.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  RM_PARITY_LOG=$O/parity.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest_gpu.log; exit 2; }
  tail -1 $O/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 3; }
  tail -1 $O/smoke.log
fi
timeout -k 10 300 python bench.py > $O/bench_C3.json 2> $O/bench_C3.err || { echo "bench C3 failed"; tail -20 $O/bench_C3.err; exit 4; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('C3 ms/step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4), 'frac', d['roofline']['frac'], 'fxaa', round(d['post_pass']['ms'],4), 'bloom', round(d['bloom_pass']['ms'],4))" $O/bench_C3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_C3 -o run -- python bench.py --cpu-seconds 0 > $O/bench_C3_under_rocprof.json 2> $O/bench_C3_under_rocprof.err || { echo "rocprof C3 failed"; exit 5; }
find $O/trace_C3 -name "*kernel_stats.csv" -exec cp {} $O/bench_C3_kernel_stats.csv \;
FRAME=random timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_fxaa_random -o run -- python tools/post_probe.py fxaa 4096 4096 20 > $O/trace_fxaa_random.log 2>&1 || { echo "fxaa noise trace failed"; exit 5; }
timeout -k 10 300 python bench.py --scene O --size 8192 --max-steps 512 --steps 5 --warmup 2 --cpu-seconds 0 > $O/bench_C5frame.json 2> $O/bench_C5frame.err || { echo "bench C5 failed"; tail -20 $O/bench_C5frame.err; exit 6; }
python -c "import json,sys; d=json.load(open(sys.argv[1])); print('C5 ms/step', round(d['ms_per_step'],4), 'kernel', round(d['kernel_ms'],4), 'frac', d['roofline']['frac'])" $O/bench_C5frame.json
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --backend gloo --cpu-seconds 0 > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { echo "gloo N=2 failed"; tail -20 $O/bench_n2_gloo.err; exit 7; }
python -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); r=d['roofline']; print('N2 gloo ms/step', round(d['ms_per_step'],4), 'frac', r['frac'], 'per_rank', r.get('per_rank_frac'), 'runs', d['balance']['runs'])" $O/bench_n2_gloo.json
if [ "${PMC:-0}" = 1 ]; then
  bash tools/pmc_profile.sh T4096$TAG || exit 8
  bash tools/pmc_profile.sh O8192$TAG --scene O --size 8192 --max-steps 512 || exit 9
  bash tools/pmc_post.sh fxaa && mv gpurun_out/pmc_fxaa $O/pmc_fxaa || exit 10
  bash tools/pmc_post.sh bloom && mv gpurun_out/pmc_bloom $O/pmc_bloom || exit 11
  bash tools/pmc_post.sh post_chain && mv gpurun_out/pmc_post_chain $O/pmc_post_chain || exit 12
  FRAME=random bash tools/pmc_post.sh fxaa && mv gpurun_out/pmc_fxaa_random $O/pmc_fxaa_random || exit 13
fi
echo "validate $TAG done"
