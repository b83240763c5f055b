set -eu
# Copy a tools/sess_final.sh run (gpurun_out/<tag>) into profiles/r05 and
# regenerate profiles/pmc_counters.json from its PMC passes.
T=$1
O=gpurun_out/$T; P=profiles/r05
for k in T4096 O8192; do
  d=gpurun_out/pmc_${k}$T
  grep '^{' $d/trace.log | tail -1 > $P/pmc_${k}${T}_bench.json
  cp $d/kernel_stats.csv $P/pmc_${k}${T}_kernel_stats.csv
  cp $d/summary.json $P/pmc_${k}${T}_summary.json
done
cp $O/bench_C3.json $P/bench_C3_$T.json
cp $O/bench_C3_kernel_stats.csv $P/bench_C3_${T}_kernel_stats.csv
cp $O/bench_C5frame.json $P/bench_C5frame_$T.json
cp $O/bench_n2_gloo.json $P/bench_n2_gloo_$T.json
cp $O/parity.jsonl $P/parity_full_size_$T.jsonl
cp $O/plugin_bench.jsonl $P/plugin_bench_$T.jsonl
cp $O/pmc_bloom/summary.json $P/pmc_bloom_${T}_summary.json
cp $O/pmc_fxaa/summary.json $P/pmc_fxaa_${T}_summary.json
cp $O/pytest_gpu.log $P/pytest_gpu_$T.log
cp $O/smoke.log $P/smoke_$T.log
{ python3 tools/bloom_trace_summary.py $O/trace_bloom_4096x4096 4096x4096
  python3 tools/bloom_trace_summary.py $O/trace_bloom_1920x1080 1920x1080; } > $P/bloom_trace_$T.jsonl
python3 tools/make_traffic_json.py $P/pmc_T4096${T}_summary.json T_4096x4096_256_P0 "rm_render_direct<1, false, 1, unsigned int>" \
  $P/pmc_T4096${T}_kernel_stats.csv "" $P/pmc_T4096${T}_bench.json > /dev/null
python3 tools/make_traffic_json.py $P/pmc_O8192${T}_summary.json O_8192x8192_512_P0 "rm_render_direct<2, false, 1, unsigned int>" \
  $P/pmc_O8192${T}_kernel_stats.csv "" $P/pmc_O8192${T}_bench.json > /dev/null
echo collected $T
