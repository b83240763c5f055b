# Decode A/B session (tools/decode_ab.py under a kernel trace, per variant library in raymarching_amd/variants/, two passes).
set -u
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for pass in 1 2; do
for v in dbase dt1 dt2 dt4 dlds; do
  RM_LIB=raymarching_amd/variants/librm_$v.so timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06l_dec/$v$pass -o run -- python tools/decode_ab.py >> gpurun_out/r06l_dec.log 2>&1 || exit 1
done
done
grep '^{' gpurun_out/r06l_dec.log
