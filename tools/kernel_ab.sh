#!/bin/bash
# GPU session: pytest -m gpu, then the render kernel timed per config with the
# hardware-dispatched tiles (auto) and persistent waves (persist), interleaved.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=$1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ge 2 ] && exit $rc
for k in auto persist auto persist; do
  RM_KERNEL=$k timeout -k 10 150 python tools/variant_bench.py raymarching_amd/librm.so >> gpurun_out/kab_$TAG.jsonl 2>> gpurun_out/kab_$TAG.err || { tail -5 gpurun_out/kab_$TAG.err; exit 3; }
done
python - "$TAG" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(f"gpurun_out/kab_{sys.argv[1]}.jsonl"):
    r = json.loads(l)
    d[(r["config"], r["kernel"], r["schedule"])].append(r["kernel_ms"])
for k in sorted(d): print(k, " ".join(f"{v:.4f}" for v in d[k]))
PY
exit $rc
