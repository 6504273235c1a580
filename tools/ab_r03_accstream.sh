#!/bin/bash
# r03: parity of the accumulate-stream + stagger build (GPU tests through OM_LIB), then an
# alternating C1 A/B of the accumulate-stream variants (tools/ablate.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03_v10}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for v in asst4; do
  OM_LIB=$PWD/_abl/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge_cases.py tests/test_multi_gpu.py -m gpu -x -q \
      --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_$v.txt" 2>&1 || { echo "pytest $v failed"; exit 1; }
  tail -1 "$OUT/pytest_$v.txt"
done
bash tools/ab.sh "$TAG/ab_accstream" "${AB:-acc8 as asst2 asst4 asmst4 asmst4 asst4 asst2 as acc8}" || exit 1
echo ok
