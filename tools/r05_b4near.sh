#!/bin/bash
# GPU box: the 4-wide traversal without the sort (nearest hit next, others pushed in slot order,
# _abl/lib_b4near.so, built from a tree with OM_BVH4_NEAREST, since removed) vs the sorted half BVH4
# and the default BVH2 on C3; bvh4 parity first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05_b4near}
mkdir -p "$OUT"
OM_LIB=$PWD/_abl/lib_b4near.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge_cases.py -m gpu -x -q \
    -k "bvh4 or ten_k" --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1 \
    || { echo "pytest failed"; tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
: > "$OUT/ab_C3.jsonl"
run() {   # variant kernel
  echo "{\"variant\": \"$1-$2\"}" >> "$OUT/ab_C3.jsonl"
  OM_LIB=$PWD/_abl/lib_$1.so timeout -k 10 200 python bench.py --config C3 --warmup 2 --no-cpu-baseline --no-window-parity \
      --kernel "$2" >> "$OUT/ab_C3.jsonl" 2>> "$OUT/ab.err" || { echo "variant $1 $2 failed"; exit 1; }
}
run base auto && run base bvh4 && run b4near bvh4 && run base auto && run base bvh4 && run b4near bvh4 || exit 1
python tools/ab_print.py "$OUT"/ab_C3.jsonl
echo ok
