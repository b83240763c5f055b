set -u
# Price of the two markers recorded when the renderer leaves a stream
# (RM_LEAVE_NO_RECORD=1, analysis only): single-stream switch probe and the
# two-stream per-rank share loop of tools/scale_model.py (C3, N = 8 shares).
O=gpurun_out/${1:-r05s}
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 200 python tools/stream_switch_probe.py > $O/switch_base_$i.jsonl 2>&1 || exit 2
  RM_LEAVE_NO_RECORD=1 timeout -k 10 200 python tools/stream_switch_probe.py > $O/switch_norec_$i.jsonl 2>&1 || exit 3
  timeout -k 10 300 python tools/scale_model.py --config C3 --ns 8 --frames 96 --even-only > $O/scale_base_$i.jsonl 2>&1 || exit 4
  RM_LEAVE_NO_RECORD=1 timeout -k 10 300 python tools/scale_model.py --config C3 --ns 8 --frames 96 --even-only > $O/scale_norec_$i.jsonl 2>&1 || exit 5
done
for f in $O/switch_*.jsonl $O/scale_*.jsonl; do echo "== $f"; grep '^{' $f | cut -c1-400; done
