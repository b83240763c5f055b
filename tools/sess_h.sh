set -u
V=raymarching_amd/variants
O=gpurun_out
POST=bloom timeout -k 10 200 python tools/post_variant_ab.py $V/librm_now.so $V/librm_bl2.so $V/librm_now.so $V/librm_bl2.so > $O/bloom_ab_r05.log 2>&1 || { tail -5 $O/bloom_ab_r05.log; exit 4; }
grep -v amdgpu.ids $O/bloom_ab_r05.log
timeout -k 10 300 python -u -m pytest tests/test_plugins.py -x -q --timeout 120 --timeout-method thread > $O/pytest_plugins_r05h.log 2>&1; rc=$?
tail -3 $O/pytest_plugins_r05h.log
[ $rc -ne 0 ] && exit $rc
for l in $V/librm_now.so raymarching_amd/librm.so; do
  RM_LIB=$l timeout -k 10 200 python tools/plugin_bench.py --reps 7 --cases 'O plugin,SC,MB' >> $O/plugkern_r05.jsonl || exit 5
done
cut -c1-160 $O/plugkern_r05.jsonl
