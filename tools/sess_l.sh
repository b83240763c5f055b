set -u
V=raymarching_amd/variants
O=gpurun_out
RM_LIB=$V/librm_nl.so RM_PARITY_LOG=$O/parity_r05l.jsonl timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "c2_1080p or c3_4096 or golden or poses or timed" > $O/pytest_r05l.log 2>&1; rc=$?
tail -3 $O/pytest_r05l.log
python -c "
import json
for l in open('$O/parity_r05l.jsonl'):
    d=json.loads(l); print(d['scene'],d['W'],d['H'], [round(s['f2e3'],7) for s in d['stats']], round(d['step_map_exact'],6))
"
[ $rc -ne 0 ] && exit $rc
CONFIGS=C3,C4share,C2P1 EQUAL=0 bash tools/ab_session.sh r05l $V/librm_new.so $V/librm_nl.so
