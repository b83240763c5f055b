#!/bin/bash
# round 3: PMC + kernel-trace profiles of the C3 and C5 render kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/pmc_profile.sh T4096r03b || exit 1
bash tools/pmc_profile.sh O8192r03 --scene O --size 8192 --max-steps 512 || exit 1
