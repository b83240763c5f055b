set -u
# FXAA short-span rows as the default: GPU tests, then FXAA time by content
O=gpurun_out/${1:-r05x3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 2; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python tools/fxaa_content_probe.py > $O/fxaa_content.jsonl 2> $O/fxaa_content.err || { tail $O/fxaa_content.err; exit 3; }
RM_LIB=raymarching_amd/variants/librm_noflat.so timeout -k 10 200 python tools/fxaa_content_probe.py > $O/fxaa_content_noflat.jsonl 2> $O/fxaa_content_noflat.err || { tail $O/fxaa_content_noflat.err; exit 3; }
cat $O/fxaa_content.jsonl $O/fxaa_content_noflat.jsonl
