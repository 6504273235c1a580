#!/bin/bash
# GPU box: parity of library variants (_abl/lib_<v>.so, tools/ablate.sh build) through OM_LIB, then
# an alternating A/B of the variants per config.
#   PARITY="v1 v2" bash tools/ab_run.sh TAG "v1 v2 v2 v1" "C1 C3" [bench args...]
#   -> gpurun_out/TAG/pytest_<v>.txt, gpurun_out/TAG/ab_<cfg>.jsonl
# PARITY_TESTS overrides the test files (default: the parity, edge-case and production-shape tests).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; VARS=$2; CFGS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
TESTS=${PARITY_TESTS:-tests/test_gpu_parity.py tests/test_gpu_edge_cases.py tests/test_gpu_production_shapes.py}
for v in $PARITY; do
  OM_LIB=$PWD/_abl/lib_$v.so timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 \
      --timeout-method thread -p no:cacheprovider > "$OUT/pytest_$v.txt" 2>&1 \
      || { echo "parity $v failed"; tail -30 "$OUT/pytest_$v.txt"; exit 1; }
  echo "parity $v: $(tail -1 "$OUT/pytest_$v.txt")"
done
for c in $CFGS; do
  : > "$OUT/ab_$c.jsonl"
  for v in $VARS; do
    echo "{\"variant\": \"$v\"}" >> "$OUT/ab_$c.jsonl"
    OM_LIB=$PWD/_abl/lib_$v.so timeout -k 10 200 python bench.py --warmup 2 --no-cpu-baseline --no-window-parity --config $c "$@" \
        >> "$OUT/ab_$c.jsonl" 2>> "$OUT/ab.err" || { echo "variant $v $c failed"; exit 1; }
  done
done
python tools/ab_print.py "$OUT"/ab_*.jsonl
echo ok
