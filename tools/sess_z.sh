set -u
# FXAA (IEEE minimum/maximum luma range, 32-bit staging offsets): parity and
# trace timing; scene-O phase ablation (shadow / SSS / reflection removed) at
# 4096^2 / 512 steps
O=gpurun_out/${1:-r05z}
V=raymarching_amd/variants
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_fxaa.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_fxaa.log 2>&1 || { tail -30 $O/pytest_fxaa.log; exit 2; }
tail -1 $O/pytest_fxaa.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_fxaa -o run -- python tools/post_probe.py fxaa 4096 4096 20 > $O/trace_fxaa.log 2>&1 || { tail -5 $O/trace_fxaa.log; exit 3; }
grep fxaa $(find $O/trace_fxaa -name "*kernel_stats.csv") | cut -d, -f1-4
for l in raymarching_amd/librm.so $V/librm_abl_sh.so $V/librm_abl_sss.so $V/librm_abl_refl.so; do RM_LIB=$l timeout -k 10 120 python tools/plugin_bench.py --reps 7 --cases 'O builtin' >> $O/ablate_O.jsonl || exit 5; done
cut -c1-140 $O/ablate_O.jsonl
