#!/bin/bash
# PC sampling (rocprofv3 beta) of the scene-O render kernel: where its waves are.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pcs
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/list.txt 2>&1 || echo "list rc=$?"
grep -i -A12 "pc_sampl\|PC Sampling" $O/list.txt | head -40
METHOD=${METHOD:-host_trap}
UNIT=${UNIT:-time}
INTERVAL=${INTERVAL:-1}
timeout -s KILL 180 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method $METHOD --pc-sampling-unit $UNIT \
  --pc-sampling-interval $INTERVAL --output-format csv -d $O/run -o run -- \
  python bench.py --scene ${SCENE:-O} --size ${SIZE:-4096} --max-steps ${STEPS:-512} --steps 5 --warmup 1 --spinup 0 --cpu-seconds 0 > $O/run.log 2>&1
rc=$?
tail -5 $O/run.log
find $O/run -type f | head
exit $rc
