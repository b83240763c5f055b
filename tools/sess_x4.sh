set -u
# FXAA pixel blocks per wave pass (RM_FXAA_BW = 32/16/8 against the 64x1 rows):
# parity of each, then FXAA time by content, and the hash A/B on the C3 frame
O=gpurun_out/${1:-r05x4}
V=raymarching_amd/variants
mkdir -p $O
export TMPDIR=/tmp
for n in bw32 bw16 bw8; do
  RM_LIB=$V/librm_$n.so timeout -k 10 300 python -u -m pytest tests/test_fxaa.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$n.log 2>&1 || { tail -30 $O/pytest_$n.log; exit 2; }
  echo "$n $(tail -1 $O/pytest_$n.log)"
done
for l in raymarching_amd/librm.so $V/librm_bw32.so $V/librm_bw16.so $V/librm_bw8.so; do
  echo "== $l" >> $O/content.log
  RM_LIB=$l timeout -k 10 200 python tools/fxaa_content_probe.py >> $O/content.log 2>/dev/null || exit 3
done
timeout -k 10 300 python tools/post_variant_ab.py raymarching_amd/librm.so $V/librm_bw32.so $V/librm_bw16.so $V/librm_bw8.so > $O/ab.log 2>&1 || exit 4
cat $O/content.log; grep fxaa_ms $O/ab.log
