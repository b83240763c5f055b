set -u
# Plugin probe instance with reassociation (RM_PROBE_REASSOC, through
# RM_PLUGIN_EXTRA_FLAGS): plugin parity with the flag, then interleaved timings.
O=gpurun_out/${1:-r05r}
mkdir -p $O
export TMPDIR=/tmp
RM_PLUGIN_EXTRA_FLAGS=-DRM_PROBE_REASSOC=1 timeout -k 10 400 python -u -m pytest tests/test_plugins.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_plugins_reassoc.log 2>&1 || { tail -30 $O/pytest_plugins_reassoc.log; exit 2; }
tail -1 $O/pytest_plugins_reassoc.log
for i in 1 2; do
  timeout -k 10 250 python tools/plugin_bench.py --reps 7 --cases 'O plugin,SC,MB' > $O/pb_base_$i.jsonl || exit 3
  RM_PLUGIN_EXTRA_FLAGS=-DRM_PROBE_REASSOC=1 timeout -k 10 250 python tools/plugin_bench.py --reps 7 --cases 'O plugin,SC,MB' > $O/pb_reassoc_$i.jsonl || exit 4
done
for f in $O/pb_*.jsonl; do echo "$f"; cut -c1-150 $f; done
