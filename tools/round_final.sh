#!/bin/bash
# End-of-round evidence on the GPU box (replaces the r02 one-off scripts):
#   tools/gpu_check.sh TAG   tests, smoke, bench, rocprofv3 kernel trace + stats, timing modes,
#                            C1 PMC passes
#   then the PMC passes of C2 (all five) and C4 (the FETCH_SIZE / WRITE_SIZE traffic passes).
#   bash tools/round_final.sh r03_final        -> gpurun_out/r03_final/...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-round_final}
bash tools/gpu_check.sh "$TAG" || exit 1
bash tools/pmc.sh "$TAG/pmcC2" --config C2 --no-extras > "gpurun_out/$TAG/pmcC2.log" 2>&1 || { echo "pmc C2 failed"; exit 1; }
PASSES="3 4" bash tools/pmc.sh "$TAG/pmcC4" --config C4 --no-extras > "gpurun_out/$TAG/pmcC4.log" 2>&1 || { echo "pmc C4 failed"; exit 1; }
echo ok
