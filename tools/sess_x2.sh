set -u
# FXAA short-span rows (RM_FXAA_FLAT): parity, then interleaved timing on the
# scene-T frame
O=gpurun_out/${1:-r05x2}
V=raymarching_amd/variants
mkdir -p $O
export TMPDIR=/tmp
RM_LIB=$V/librm_fxflat.so timeout -k 10 300 python -u -m pytest tests/test_fxaa.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_fxflat.log 2>&1 || { tail -30 $O/pytest_fxflat.log; exit 2; }
tail -1 $O/pytest_fxflat.log
L="raymarching_amd/librm.so $V/librm_fxflat.so"
for i in 1 2 3; do timeout -k 10 300 python tools/post_variant_ab.py $L >> $O/fxaa_flat_ab.log 2>&1 || { tail $O/fxaa_flat_ab.log; exit 3; }; done
grep fxaa_ms $O/fxaa_flat_ab.log
