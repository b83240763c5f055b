#!/bin/bash
# Build librm.so A/B variants for tools/variant_bench.py: one per RM_OPT mask
# (rm_device.h), each in its own build directory, into raymarching_amd/variants/.
# Usage: tools/build_variants.sh MASK [MASK ...]
set -eu
cd "$(dirname "$0")/../raymarching_amd"
mkdir -p variants
for m in "$@"; do
  make -s B=build/opt$m LIB=variants/librm_opt$m.so EXTRA=-DRM_OPT=$m variants/librm_opt$m.so -j8
done
ls -la variants
