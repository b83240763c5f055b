#!/bin/bash
# PMC passes (one rocprofv3 run per counter group, no tracing domains) over any
# python command; summaries via tools/pmc_parse.py -> DIR/summary.json.
# Usage: bash tools/pmc_any.sh DIR python-script [args...]
set -u
export TMPDIR=/tmp
D=$1; shift
mkdir -p $D
i=0
while read -r G; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --output-format csv -d $D/p$i -o run -- python "$@" > $D/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU
SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS
FETCH_SIZE
WRITE_SIZE
GROUPS
python tools/pmc_parse.py $D > $D/summary.json
