#!/bin/bash
# r04 late: every GPU test + the full bench line (with configs.C1_adaptive) on the final build,
# then the adaptive schedules at 512 spp in 128-spp calls (production build timed).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_quick.sh r04_q6 "" || exit 1
timeout -k 10 300 python tools/adaptive_bench.py 128 C1 512 > gpurun_out/r04_q6/adaptive_512.json || exit 1
cat gpurun_out/r04_q6/adaptive_512.json
echo ok
