set -u
V=raymarching_amd/variants
O=gpurun_out
POST=bloom timeout -k 10 200 python tools/post_variant_ab.py $V/librm_now.so $V/librm_bl2.so $V/librm_now.so $V/librm_bl2.so > $O/bloom_ab_r05.log 2>&1 || { tail -5 $O/bloom_ab_r05.log; exit 4; }
grep -v amdgpu.ids $O/bloom_ab_r05.log
timeout -k 10 200 python tools/post_variant_ab.py $V/librm_now.so > $O/fxaa_now_r05.log 2>&1 || exit 5
grep -v amdgpu.ids $O/fxaa_now_r05.log
