#!/bin/bash
# End-of-round evidence on the GPU box: tools/gpu_check.sh (tests, smoke, bench, rocprofv3
# kernel trace + stats, timing modes, C1 PMC passes), then the C2 / C3 PMC traffic passes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r02_final}
bash tools/gpu_check.sh "$TAG" || exit 1
bash tools/pmc.sh "$TAG/pmcC2" --config C2 --no-extras > "gpurun_out/$TAG/pmcC2.log" 2>&1 || { echo "pmc C2 failed"; exit 1; }
bash tools/pmc.sh "$TAG/pmcC3" --config C3 --no-extras > "gpurun_out/$TAG/pmcC3.log" 2>&1 || { echo "pmc C3 failed"; exit 1; }
echo ok
