#!/bin/bash
# r04 late: GPU tests on the variable adaptive batches, then the later-batch A/B (C1 512 spp in
# 128-spp calls, and 64 spp in one call).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_q5; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "adaptive or concurrent or auto_pipeline" > $OUT/pytest_gpu.txt 2>&1 || { tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
bash tools/ab_adaptive.sh r04_q5 "base al32 al64 base al32 al64" 128 C1 512 || exit 1
bash tools/ab_adaptive.sh r04_q5b "base al64 base al64" 64 C1 64 || exit 1
echo ok
