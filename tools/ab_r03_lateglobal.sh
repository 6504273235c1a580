#!/bin/bash
# r03: late bounces reading the BVH2 through the caches (OM_WF_LATE_GLOBAL): parity of one build
# through OM_LIB, then an alternating C1 A/B (tools/ablate.sh variants).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03_v11}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
OM_LIB=$PWD/_abl/lib_lg6.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge_cases.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_lg6.txt" 2>&1 || { echo "pytest lg6 failed"; exit 1; }
tail -1 "$OUT/pytest_lg6.txt"
bash tools/ab.sh "$TAG/ab_lateglobal" "base lg6 lg9 lg12 lg12 lg9 lg6 base" || exit 1
echo ok
