#!/bin/bash
# One GPU A/B session: (optional) pytest -m gpu on the default build, bit-identity
# of the variant libraries (tools/lib_equal.py), then the render kernel timed per
# config for each variant, twice interleaved (tools/variant_bench.py).
# Usage: [PYTEST=1] [SCENES=T] [CONFIGS=C3,C4share] tools/ab_session.sh TAG lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=$1; shift
if [ "${PYTEST:-0}" = 1 ]; then
  RM_PARITY_LOG=gpurun_out/parity_$TAG.jsonl timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_$TAG.log
  [ $rc -ne 0 ] && { echo "pytest rc=$rc: stopping"; exit $rc; }
fi
if [ "${EQUAL:-1}" = 1 ]; then
  timeout -k 10 400 python tools/lib_equal.py "$@" > gpurun_out/equal_$TAG.log 2>&1 || { echo "lib_equal failed"; tail -20 gpurun_out/equal_$TAG.log; exit 3; }
  tail -${EQUAL_TAIL:-8} gpurun_out/equal_$TAG.log
fi
timeout -k 10 ${VB_TIMEOUT:-600} python tools/variant_bench.py "$@" "$@" > gpurun_out/ab_$TAG.jsonl 2> gpurun_out/ab_$TAG.err || { tail -5 gpurun_out/ab_$TAG.err; exit 4; }
python - "$TAG" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(f"gpurun_out/ab_{sys.argv[1]}.jsonl"):
    r = json.loads(l)
    if r["schedule"] == 1: d[(r["config"], r["lib"])].append(r["kernel_ms"])
for k in sorted(d): print(k, " ".join(f"{v:.4f}" for v in d[k]))
PY
