#!/bin/bash
# One GPU session: gpu tests, bench, rocprofv3 kernel-trace profile of the bench.
# Stops at the first crash/timeout (exit code >= 2 from pytest, or any bench failure).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r01}
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu_$TAG.log 2>&1
rc=$?
tail -5 gpurun_out/pytest_gpu_$TAG.log
if [ $rc -ge 2 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { echo "bench failed"; tail -20 gpurun_out/bench_$TAG.err; exit 3; }
cat gpurun_out/bench_$TAG.json
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py --cpu-seconds 0 --steps 10 ${BENCH_ARGS:-} > gpurun_out/bench_prof_$TAG.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/bench_prof_$TAG.log; exit 4; }
find gpurun_out/prof_$TAG -name "*stats*" | head
exit $rc
