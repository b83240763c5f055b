# Decode A/B session (tools/decode_ab.py under a kernel trace, per variant library in raymarching_amd/variants/, two passes).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for pass in 1 2; do
for v in ${DEC_VARIANTS:-dbase}; do
  RM_LIB=raymarching_amd/variants/librm_$v.so timeout -k 10 120 python tools/decode_ab.py >> gpurun_out/${DEC_TAG:-dec}.log 2>&1 || exit 1
done
done
grep '^{' gpurun_out/${DEC_TAG:-dec}.log
