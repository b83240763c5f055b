set -u
# Round-5 final validation: tools/gpu_validate.sh (tests, smoke, C3/C5/N=2
# lines, PMC) then the plugin decomposition against the span/settle ablations.
V=raymarching_amd/variants
O=gpurun_out/$1
PMC=1 bash tools/gpu_validate.sh $1 || exit $?
for l in raymarching_amd/librm.so $V/librm_nospan.so $V/librm_nsns.so; do RM_LIB=$l timeout -k 10 120 python tools/plugin_bench.py --reps 9 --cases 'O builtin' >> $O/plugdecomp.jsonl || exit 12; done
timeout -k 10 200 python tools/plugin_bench.py --reps 9 --cases 'O plugin,SC,MB' >> $O/plugdecomp.jsonl || exit 13
cut -c1-200 $O/plugdecomp.jsonl
