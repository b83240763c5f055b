#!/bin/bash
# round 3: PMC refresh after the backface skip (C3, C5), then the bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/pmc_profile.sh T4096r03c || exit 1
bash tools/pmc_profile.sh O8192r03b --scene O --size 8192 --max-steps 512 || exit 1
