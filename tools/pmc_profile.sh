#!/bin/bash
# rocprofv3 PMC passes (one counter group per run, no tracing domains) plus one
# kernel-trace run of the same short bench command; summaries ->
# gpurun_out/pmc_<tag>/.  Usage: pmc_profile.sh TAG [bench args]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
export TMPDIR=/tmp
OUT=gpurun_out/pmc_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
    python bench.py --steps 10 --warmup 2 --cpu-seconds 0 "$@" > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
i=0
while read -r GROUP; do
  [ -z "$GROUP" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $GROUP --output-format csv -d $OUT/p$i -o run -- \
      python bench.py --steps 10 --warmup 2 --cpu-seconds 0 "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU
SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH
FETCH_SIZE
WRITE_SIZE
GROUPS
python tools/pmc_parse.py $OUT > $OUT/summary.json && find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \; && echo "pmc $TAG ok"
