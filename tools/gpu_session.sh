#!/bin/bash
# One GPU session of named steps, each under its own time limit; the first
# failing step ends the session (exit code = 10 + step index).  Steps:
#   ab:TAG:SCENES:CONFIGS:lib1,lib2,...   render-kernel A/B (tools/ab_session.sh)
#   post:TAG:POST:FRAME:lib1,lib2,...     post-pass A/B (tools/post_variant_ab.py)
#   validate:TAG[:PMC]                    round validation (tools/gpu_validate.sh)
#   cmd:TAG:SECONDS:command ...           any command, output to gpurun_out/TAG.log
# Usage: tools/gpu_session.sh STEP [STEP ...]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for step in "$@"; do
  i=$((i + 1))
  IFS=: read -r kind tag a b c <<< "$step"
  echo "== step $i: $step"
  case $kind in
    ab)
      SCENES=$a CONFIGS=$b bash tools/ab_session.sh "$tag" $(echo "$c" | tr ',' ' ') || exit $((10 + i)) ;;
    post)
      POST=$a FRAME=$b timeout -k 10 300 python tools/post_variant_ab.py $(echo "$c" | tr ',' ' ') \
        > gpurun_out/post_$tag.log 2>&1 || { tail -5 gpurun_out/post_$tag.log; exit $((10 + i)); }
      grep -v amdgpu.ids gpurun_out/post_$tag.log ;;
    validate)
      PMC=${a:-0} bash tools/gpu_validate.sh "$tag" || exit $((10 + i)) ;;
    cmd)
      rest=${step#cmd:$tag:$a:}
      timeout -k 10 "$a" bash -c "$rest" > gpurun_out/$tag.log 2>&1 || { tail -20 gpurun_out/$tag.log; exit $((10 + i)); }
      tail -20 gpurun_out/$tag.log ;;
    *) echo "unknown step $kind"; exit 2 ;;
  esac
done
echo "session done"
