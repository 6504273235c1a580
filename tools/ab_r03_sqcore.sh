#!/bin/bash
# r03: wave-uniform sqrt core in the march SDFs (OM_MARCH_SQRT_CORE): marched parity through
# OM_LIB, then an alternating C2 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03_v12}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
OM_LIB=$PWD/_abl/lib_sqcore.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge_cases.py -m gpu -x -q \
    --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_sqcore.txt" 2>&1 || { echo "pytest sqcore failed"; exit 1; }
tail -1 "$OUT/pytest_sqcore.txt"
bash tools/ab.sh "$TAG/ab_sqcore_C2" "base sqcore sqcore base base sqcore" --config C2 || exit 1
echo ok
