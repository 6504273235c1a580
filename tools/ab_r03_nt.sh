#!/bin/bash
# r03: non-temporal hints on the path-state loads/stores: parity through OM_LIB, then an
# alternating C1 A/B (tools/ablate.sh variants).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03_v13}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
OM_LIB=$PWD/_abl/lib_ntls.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge_cases.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_ntls.txt" 2>&1 || { echo "pytest ntls failed"; exit 1; }
tail -1 "$OUT/pytest_ntls.txt"
bash tools/ab.sh "$TAG/ab_nt" "base ntl nts ntls ntls nts ntl base" || exit 1
echo ok
