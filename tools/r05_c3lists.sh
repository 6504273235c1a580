#!/bin/bash
# GPU box: C3 bounce 0 with the primary-ray tile lists forced on vs AUTO (which leaves them off
# above 12 candidates per pixel), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05_c3lists}
mkdir -p "$OUT"
: > "$OUT/ab_C3.jsonl"
for r in 1 2; do
  for v in auto on; do
    echo "{\"variant\": \"lists-$v\"}" >> "$OUT/ab_C3.jsonl"
    timeout -k 10 200 python bench.py --config C3 --warmup 2 --no-cpu-baseline --primary-lists $v \
        >> "$OUT/ab_C3.jsonl" 2>> "$OUT/ab.err" || { echo "variant $v failed"; exit 1; }
  done
done
python tools/ab_print.py "$OUT"/ab_C3.jsonl
grep -o '"bit_exact_vs_oracle": [a-z]*' "$OUT"/ab_C3.jsonl | sort | uniq -c
echo ok
