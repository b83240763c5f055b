set -u
V=raymarching_amd/variants
O=gpurun_out
timeout -k 10 200 python tools/post_variant_ab.py $V/librm_cur.so $V/librm_fxA.so $V/librm_fxB.so $V/librm_fxB16.so $V/librm_cur.so $V/librm_fxB.so > $O/fxaa_ab2_r05.log 2>&1 || { tail -5 $O/fxaa_ab2_r05.log; exit 4; }
grep -v amdgpu.ids $O/fxaa_ab2_r05.log
for f in "" "-fno-hip-fp32-correctly-rounded-divide-sqrt" "-fno-hip-fp32-correctly-rounded-divide-sqrt -ffp-contract=fast"; do
  RM_PLUGIN_EXTRA_FLAGS="$f" timeout -k 10 120 python tools/plugin_bench.py --reps 7 --cases 'O plugin' | sed "s/^/flags=[$f] /" >> $O/plugflags_r05.jsonl || exit 5
done
cut -c1-220 $O/plugflags_r05.jsonl
