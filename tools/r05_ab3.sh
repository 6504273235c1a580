#!/bin/bash
# GPU box: parity of the in-tree build (OM_LIB unset), then alternating A/B of _abl/lib_<v>.so
# variants on the given configs.   bash tools/r05_ab3.sh TAG "v1 v2 ..." "C1 C3"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; VARS=$2; CFGS=$3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
for c in $CFGS; do
  : > "$OUT/ab_$c.jsonl"
  for r in 1 2; do
    for v in $VARS; do
      echo "{\"variant\": \"$v\"}" >> "$OUT/ab_$c.jsonl"
      OM_LIB=$PWD/_abl/lib_$v.so timeout -k 10 200 python bench.py --config $c --warmup 2 --no-cpu-baseline --no-window-parity \
          >> "$OUT/ab_$c.jsonl" 2>> "$OUT/ab.err" || { echo "variant $v $c failed"; exit 1; }
    done
  done
done
python tools/ab_print.py "$OUT"/ab_*.jsonl
echo ok
