set -u
V=raymarching_amd/variants
O=gpurun_out
timeout -k 10 60 ./tools/rcp_exhaustive 0.00390625 4.0 > $O/rcp_exhaustive_r05.json || exit 3
cat $O/rcp_exhaustive_r05.json
timeout -k 10 200 python tools/post_variant_ab.py $V/librm_cur.so $V/librm_fxaddr.so $V/librm_fxf4.so $V/librm_fxf4t16.so $V/librm_cur.so > $O/fxaa_ab_r05.log 2>&1 || { tail -5 $O/fxaa_ab_r05.log; exit 4; }
cat $O/fxaa_ab_r05.log
for l in cur nospan nsns; do RM_LIB=$V/librm_$l.so timeout -k 10 120 python tools/plugin_bench.py --reps 9 --cases 'O builtin' >> $O/plugdecomp_r05.jsonl || exit 5; done
RM_LIB=$V/librm_cur.so timeout -k 10 200 python tools/plugin_bench.py --reps 9 --cases 'O plugin,SC,MB' >> $O/plugdecomp_r05.jsonl || exit 6
cut -c1-200 $O/plugdecomp_r05.jsonl
