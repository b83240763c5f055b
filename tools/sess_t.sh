set -u
# One marker per stream leave (schedule entries borrow `done`): GPU tests, then
# the two-stream share loop against the marker-free analysis knob.
O=gpurun_out/${1:-r05t}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 2; }
tail -1 $O/pytest_gpu.log
for i in 1 2; do
  for v in 0 1; do
    RM_LEAVE_NO_RECORD=$v timeout -k 10 300 python tools/scale_model.py --config C3 --ns 8 --frames 96 --even-only > $O/scale_v${v}_$i.jsonl 2>&1 || exit 4
  done
done
timeout -k 10 200 python tools/stream_switch_probe.py > $O/switch.jsonl 2>&1 || exit 5
timeout -k 10 200 python tools/stream_switch_probe.py 2048 100 >> $O/switch.jsonl 2>&1 || exit 5
for f in $O/scale_*.jsonl; do echo "== $f"; grep '^{' $f | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['per_rank_frame_ms'])"; done
grep '^{' $O/switch.jsonl
