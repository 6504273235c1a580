#!/bin/bash
# r03: smaller batches on C1 (8 / 12 spp per batch, two streams), 128 and 96 spp per call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03_v15}
bash tools/ab.sh "$TAG/ab_bs8_128" "base bs8 bs8 base" || exit 1
bash tools/ab.sh "$TAG/ab_bs12_96" "base bs12 bs12 base" --spp-per-step 96 --steps 6 || exit 1
echo ok
