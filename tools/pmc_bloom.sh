set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcb
i=0
while read -r G; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $G --output-format csv -d gpurun_out/pmcb/p$i -o run -- python tools/bloom_probe.py 4096 4096 5 > gpurun_out/pmcb/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done <<'GROUPS'
SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_SALU
SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VMEM_RD SQ_INSTS_LDS
GROUPS
