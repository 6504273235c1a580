#!/bin/bash
# GPU box: the in-tree build (slab min/max as IEEE minimum/maximum, no per-visit canonicalise; no
# stack-depth guard) -- full -m gpu suite, then alternating A/B vs _abl/lib_base.so on C1-C4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05_mm}
mkdir -p "$OUT"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
for c in ${CFGS:-C1 C3 C2 C4}; do
  : > "$OUT/ab_$c.jsonl"
  for v in base mm base mm; do
    echo "{\"variant\": \"$v\"}" >> "$OUT/ab_$c.jsonl"
    OM_LIB=$PWD/_abl/lib_$v.so timeout -k 10 200 python bench.py --config $c --warmup 2 --no-cpu-baseline --no-window-parity \
        >> "$OUT/ab_$c.jsonl" 2>> "$OUT/ab.err" || { echo "variant $v $c failed"; exit 1; }
  done
done
python tools/ab_print.py "$OUT"/ab_*.jsonl
echo ok
