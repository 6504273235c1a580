#!/bin/bash
# r04 late check: GPU tests + full bench line, then the C2 tail/segment A/B and the adaptive batch A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
bash tools/gpu_quick.sh r04_q3 "" || exit 1
python tools/ab_print.py gpurun_out/r04_q3/bench.json
NO_TESTS=1 bash tools/ab_quick.sh r04_q3 "base tsh4 tsh16 mu12 mlpc4k mlpc16k tm0 tm0l16 base tsh4 tsh16 mu12 mlpc4k mlpc16k tm0 tm0l16" "C2" || exit 1
bash tools/ab_adaptive.sh r04_q3 "base ab8 base ab8" 64 C1 || exit 1
echo ok
