#!/bin/bash
# GPU box: leaf sphere records through sphere_root_diag (axis-aligned spheres, wave-uniform choice)
# vs the previous build (_abl/lib_base.so) and a forced-diagonal build (_abl/lib_diagonly.so, wrong
# answers on rotated spheres). Both variants were built from an uncommitted tree and removed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05_diag}
mkdir -p "$OUT"
OM_LIB=$PWD/_abl/lib_diag.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edge_cases.py -m gpu -x -q \
    --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_diag.txt" 2>&1 \
    || { echo "pytest diag failed"; tail -30 "$OUT/pytest_diag.txt"; exit 1; }
tail -1 "$OUT/pytest_diag.txt"
for c in ${CFGS:-C1 C3}; do
  : > "$OUT/ab_$c.jsonl"
  for v in base diag diagonly base diag diagonly; do
    echo "{\"variant\": \"$v\"}" >> "$OUT/ab_$c.jsonl"
    OM_LIB=$PWD/_abl/lib_$v.so timeout -k 10 200 python bench.py --config $c --warmup 2 --no-cpu-baseline \
        >> "$OUT/ab_$c.jsonl" 2>> "$OUT/ab.err" || { echo "variant $v $c failed"; exit 1; }
  done
done
python tools/ab_print.py "$OUT"/ab_*.jsonl
grep -o '"bit_exact_vs_oracle": [a-z]*' "$OUT"/ab_*.jsonl | sort | uniq -c
echo ok
