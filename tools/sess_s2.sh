set -u
# Which of the two leave markers costs (RM_LEAVE_NO_RECORD=2: schedule
# entries' records skipped; =3: `done` skipped; analysis only)
O=gpurun_out/${1:-r05s2}
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  for v in 0 2 3 1; do
    RM_LEAVE_NO_RECORD=$v timeout -k 10 300 python tools/scale_model.py --config C3 --ns 8 --frames 96 --even-only > $O/scale_v${v}_$i.jsonl 2>&1 || exit 4
  done
done
for f in $O/scale_*.jsonl; do echo "== $f"; grep '^{' $f | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print(d['per_rank_frame_ms'])"; done
