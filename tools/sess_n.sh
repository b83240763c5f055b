set -u
V=raymarching_amd/variants
O=gpurun_out
RM_PARITY_LOG=$O/parity_r05n.jsonl timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_r05n.log 2>&1; rc=$?
tail -3 $O/pytest_r05n.log
python -c "
import json
for l in open('$O/parity_r05n.jsonl'):
    d=json.loads(l); print(d['scene'],d['W'],d['H'], [round(s['f2e3'],7) for s in d['stats']], [round(s['max'],6) for s in d['stats']], round(d['step_map_exact'],6))
"
[ $rc -ne 0 ] && exit $rc
CONFIGS=O4096,C5frame,C5share EQUAL=0 bash tools/ab_session.sh r05n $V/librm_oc.so $V/librm_fc.so
for l in $V/librm_oc.so $V/librm_fc.so; do RM_LIB=$l timeout -k 10 200 python tools/plugin_bench.py --reps 7 --cases 'O plugin' >> $O/plugfc_r05.jsonl || exit 5; done
cut -c1-150 $O/plugfc_r05.jsonl
