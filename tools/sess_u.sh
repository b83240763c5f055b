set -u
# Kept streams (rm_set_stream_kept: no marker per leave): GPU tests, then the
# two-stream share loop, plain vs kept vs the marker-free analysis knob.
O=gpurun_out/${1:-r05u}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 2; }
tail -1 $O/pytest_gpu.log
for i in 1 2; do
  timeout -k 10 300 python tools/scale_model.py --config C3 --ns 8 --frames 96 --even-only > $O/scale_plain_$i.jsonl 2>&1 || exit 4
  timeout -k 10 300 python tools/scale_model.py --config C3 --ns 8 --frames 96 --even-only --kept > $O/scale_kept_$i.jsonl 2>&1 || exit 4
  RM_LEAVE_NO_RECORD=1 timeout -k 10 300 python tools/scale_model.py --config C3 --ns 8 --frames 96 --even-only > $O/scale_none_$i.jsonl 2>&1 || exit 4
done
for f in $O/scale_*.jsonl; do echo "== $f"; grep '^{' $f | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['per_rank_frame_ms'])"; done
