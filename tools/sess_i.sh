set -u
V=raymarching_amd/variants
O=gpurun_out
POST=bloom timeout -k 10 200 python tools/post_variant_ab.py $V/librm_nw.so $V/librm_bw6.so $V/librm_bw8.so $V/librm_nw.so $V/librm_bw6.so $V/librm_bw8.so > $O/bloom_ab2_r05.log 2>&1 || { tail -5 $O/bloom_ab2_r05.log; exit 4; }
grep -v amdgpu.ids $O/bloom_ab2_r05.log
SCENES=O,OG CONFIGS=O4096,C5frame,C5share EQUAL_TAIL=3 bash tools/ab_session.sh r05i $V/librm_nw.so $V/librm_ou.so
