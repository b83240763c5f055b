set -u
# Round-end validation on one GPU box: tools/gpu_validate.sh with PMC (GPU
# tests, smoke, C3 line + kernel trace, C5 line, gloo N=2, PMC of C3/C5 and the
# post passes), then the bloom kernel traces and the plugin timings.
TAG=$1
O=gpurun_out/$TAG
PMC=1 bash tools/gpu_validate.sh $TAG || exit $?
for sz in "4096 4096" "1920 1080"; do
  t=$(echo $sz | tr ' ' x)
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_bloom_$t -o run -- python tools/post_probe.py bloom $sz 20 > $O/trace_bloom_$t.log 2>&1 || exit 12
done
timeout -k 10 250 python tools/plugin_bench.py --reps 9 --cases 'O builtin,O plugin,SC,MB' > $O/plugin_bench.jsonl || exit 13
cut -c1-160 $O/plugin_bench.jsonl
echo "final $TAG done"
