set -u
# FXAA occupancy variants: halo 4 + lumas only where the +-1 taps read them
# (LDS 24.9 -> 20.5 KB), 4 or 8 waves per workgroup, 16/32/64-row tiles.
# Parity of each variant (tests/test_fxaa.py, RM_LIB) and interleaved timing.
O=gpurun_out/${1:-r05q}
V=raymarching_amd/variants
mkdir -p $O
export TMPDIR=/tmp
for n in fxh4t fxh4t8 fxh4t8y64 fxh4t16; do
  RM_LIB=$V/librm_$n.so timeout -k 10 300 python -u -m pytest tests/test_fxaa.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_$n.log 2>&1 || { tail -30 $O/pytest_$n.log; exit 2; }
  echo "$n $(tail -1 $O/pytest_$n.log)"
done
L="raymarching_amd/librm.so $V/librm_fxh4t.so $V/librm_fxh4t8.so $V/librm_fxh4t8y64.so $V/librm_fxh4t16.so $V/librm_fxh4t8r4.so"
timeout -k 10 300 python tools/post_variant_ab.py $L > $O/fxaa_occ_ab.log 2>&1 || { tail $O/fxaa_occ_ab.log; exit 3; }
timeout -k 10 300 python tools/post_variant_ab.py $L >> $O/fxaa_occ_ab.log 2>&1 || { tail $O/fxaa_occ_ab.log; exit 3; }
grep fxaa_ms $O/fxaa_occ_ab.log
