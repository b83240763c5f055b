#!/bin/bash
# A/B of RM_LAT_TILES values on the current librm.so
cd "${GRAFT_REPO_ROOT:-.}"
for n in ${LAT_LIST:-0 1024 2048 4096 8192}; do
  RM_LAT_TILES=$n CONFIGS=C3,C4share,C2P1 timeout -k 10 200 python tools/variant_bench.py raymarching_amd/librm.so 2>/dev/null | grep '"schedule": 1' | sed "s/^{/{\"lat\": $n, /" || exit 1
done
