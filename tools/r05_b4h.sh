#!/bin/bash
# GPU box: half-precision BVH4 through L2 (OM_KERNEL_BVH4 on S-10k) vs the default BVH2 on C3,
# parity first, then alternating bench runs and the LDS-prefix variants (_abl/lib_h4p*.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05_b4h}
mkdir -p "$OUT" _abl
cp raytracingoneweekend_amd/libottomarcher.so _abl/lib_base.so
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge_cases.py tests/test_golden.py -m gpu -x -q \
    -k "bvh4 or ten_k" --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.txt" 2>&1 \
    || { echo "pytest failed"; tail -30 "$OUT/pytest.txt"; exit 1; }
tail -1 "$OUT/pytest.txt"
: > "$OUT/ab_C3.jsonl"
run() {   # variant kernel
  echo "{\"variant\": \"$1-$2\"}" >> "$OUT/ab_C3.jsonl"
  OM_LIB=$PWD/_abl/lib_$1.so timeout -k 10 200 python bench.py --config C3 --warmup 2 --no-cpu-baseline --no-window-parity \
      --kernel "$2" >> "$OUT/ab_C3.jsonl" 2>> "$OUT/ab.err" || { echo "variant $1 $2 failed"; exit 1; }
}
run base auto && run base bvh4 && run base auto && run base bvh4 && \
  run h4p0 bvh4 && run h4p4k bvh4 && run h4p12k bvh4 && run base bvh4 && run base auto || exit 1
python tools/ab_print.py "$OUT"/ab_C3.jsonl
echo ok
