# PMC passes (one rocprofv3 run per counter group) over tools/post_probe.py.
# Usage: [FRAME=random] bash tools/pmc_post.sh fxaa|bloom|post_chain ; summaries via
# tools/pmc_parse.py -> gpurun_out/pmc_<which>[_random]/summary.json
set -u
export TMPDIR=/tmp
P=${1:-fxaa}
D=gpurun_out/pmc_$P${FRAME:+_$FRAME}
mkdir -p $D
i=0
while read -r G; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G --output-format csv -d $D/p$i -o run -- python tools/post_probe.py $P 4096 4096 5 > $D/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU
SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT
FETCH_SIZE
WRITE_SIZE
GROUPS
python tools/pmc_parse.py $D > $D/summary.json
