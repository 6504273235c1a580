#!/bin/bash
# End-of-round evidence on the GPU box:
#   tools/gpu_check.sh TAG   tests, smoke, bench, rocprofv3 kernel trace + stats, timing modes
#   tools/pmc_final.sh       the PMC passes of C1 and C2 (all five) and C4 (FETCH_SIZE / WRITE_SIZE),
#                            summarised on the box (the raw counter files exceed gpurun's 64 MiB return)
#   bash tools/round_final.sh r03_final        -> gpurun_out/r03_final/..., gpurun_out/r03_final_pmc/...
# (Two gpurun calls fit the 20-minute limit better: NO_PMC=1 tools/gpu_check.sh, then tools/pmc_final.sh.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-round_final}
NO_PMC=1 bash tools/gpu_check.sh "$TAG" || exit 1
bash tools/pmc_final.sh "${TAG}_pmc" || { echo "pmc failed"; exit 1; }
echo ok
