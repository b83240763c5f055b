#!/bin/bash
# Build librm.so A/B variants for tools/variant_bench.py: each NAME=FLAGS pair
# (extra device-compile flags, e.g. experiment macros) in its own build
# directory, into raymarching_amd/variants/librm_NAME.so.
# Usage: tools/build_variants.sh NAME='-DFOO=1 -DBAR' [NAME=FLAGS ...]
set -eu
cd "$(dirname "$0")/../raymarching_amd"
mkdir -p variants
for spec in "$@"; do
  name=${spec%%=*}; flags=${spec#*=}
  make -s B=build/v_$name LIB=variants/librm_$name.so EXTRA="$flags" variants/librm_$name.so -j8
done
ls -la variants
