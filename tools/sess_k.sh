set -u
V=raymarching_amd/variants
O=gpurun_out
RM_PARITY_LOG=$O/parity_r05k.jsonl timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_accumulate.py -x -q --timeout 200 --timeout-method thread > $O/pytest_r05k.log 2>&1; rc=$?
tail -3 $O/pytest_r05k.log
[ $rc -ne 0 ] && exit $rc
python -c "
import json
for l in open('$O/parity_r05k.jsonl'):
    d=json.loads(l); print(d['scene'],d['W'],d['H'],d['pose'].get('time') if isinstance(d['pose'],dict) else '', [round(s['f2e3'],7) for s in d['stats']], round(d['step_map_exact'],6))
"
CONFIGS=C3,C4share,C2P1 EQUAL=0 bash tools/ab_session.sh r05k $V/librm_old.so $V/librm_new.so
