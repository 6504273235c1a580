#!/bin/bash
# r03: parity of the merged-late-bounce and grouped-accumulate builds (GPU tests through OM_LIB),
# then an alternating C1 A/B of them (tools/ablate.sh variants), then C3 BVH4 and the C2 tail sweep.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03_v9}
mkdir -p "$OUT"
for v in m6f8 acc8m8f4; do
  OM_LIB=$PWD/_abl/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge_cases.py -m gpu -x -q \
      --timeout 200 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_$v.txt" 2>&1 || { echo "pytest $v failed"; exit 1; }
  tail -1 "$OUT/pytest_$v.txt"
done
bash tools/ab.sh "${1:-r03_v9}/ab_merge" "base m8f4 m6f4 m6f8 m10f8 acc8 acc8m8f4 acc8m8f4 acc8 m10f8 m6f8 m6f4 m8f4 base" || exit 1
bash tools/ab_kernel_c3.sh || exit 1
echo ok
