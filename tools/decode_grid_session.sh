# Decode grid-cap A/B (tools/; not product): per variant library, the root
# decode alone (tools/decode_ab.py) and the N = 8 frame model whose root frames
# decode inside the frame loop (tools/scale_model.py --wire delta).
set -u
cd $GRAFT_REPO_ROOT
for v in ${DEC_VARIANTS:-gy0}; do
  echo "== $v"
  RM_LIB=raymarching_amd/variants/librm_$v.so DEC_NS=8 timeout -k 10 120 python tools/decode_ab.py 2>/dev/null | grep '^{' || exit 1
  RM_LIB=raymarching_amd/variants/librm_$v.so timeout -k 10 200 python tools/scale_model.py --config C3 --ns 8 --wire delta --kept --even-only 2>/dev/null | grep '^{' || exit 1
done
