#!/bin/bash
# GPU A/B session: pytest -m gpu on the default build, then tools/variant_bench.py
# over the given variant libraries (twice, interleaved).  Usage:
#   CONFIGS=C3,C4share tools/ab_run.sh TAG lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_$TAG.log
[ $rc -ge 2 ] && exit $rc
timeout -k 10 600 python tools/variant_bench.py "$@" "$@" > gpurun_out/ab_$TAG.jsonl 2> gpurun_out/ab_$TAG.err || { tail -5 gpurun_out/ab_$TAG.err; exit 3; }
python - "$TAG" <<'PY'
import json, sys, collections
d = collections.defaultdict(list)
for l in open(f"gpurun_out/ab_{sys.argv[1]}.jsonl"):
    r = json.loads(l)
    if r["schedule"] == 1: d[(r["config"], r["lib"])].append(r["kernel_ms"])
for k in sorted(d): print(k, " ".join(f"{v:.4f}" for v in d[k]))
PY
exit $rc
