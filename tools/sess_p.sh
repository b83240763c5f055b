set -u
# plugin O phase ablation (RM_PLUGIN_EXTRA_FLAGS: the plugin translation unit's
# own macros) beside the built-in's (variant libraries), 4096^2 / 512 steps
O=gpurun_out/${1:-r05p}
mkdir -p $O
for f in "" "-DRM_ABLATE_SHADOW" "-DRM_ABLATE_SSS" "-DRM_ABLATE_SHADOW -DRM_ABLATE_SSS"; do
  RM_PLUGIN_EXTRA_FLAGS="$f" timeout -k 10 150 python tools/plugin_bench.py --reps 7 --cases 'O plugin' | sed "s/^{/{\"flags\": \"$f\", /" >> $O/plugin_ablate.jsonl || exit 5
done
python -c "
import json
for l in open('$O/plugin_ablate.jsonl'):
    d=json.loads(l); print(repr(d['flags']), d['kernel_ms'])
"
