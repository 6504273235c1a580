#!/bin/bash
# r04 end: the full -m gpu suite and smoke on the final tree, then the C1/C2/C3 batch-size A/B
# (OM_WF_MIN_PATHS_LOG2 = 26: 32-spp batches at 1080p).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_end; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.txt 2>&1 || { tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
NO_TESTS=1 bash tools/ab_quick.sh r04_end "base mn26 base mn26" "C1 C3 C2" || exit 1
echo ok
