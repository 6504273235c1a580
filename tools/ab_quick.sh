#!/bin/bash
# GPU box: the -m gpu tests on the in-tree build, then an alternating A/B of library builds
# (_abl/lib_<v>.so, e.g. a baseline from an earlier commit) per config.
#   bash tools/ab_quick.sh TAG "v1 v2 v2 v1" "C1 C3" [bench args...]   -> gpurun_out/TAG/ab_<cfg>.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; VARS=$2; CFGS=$3; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
      > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
  tail -1 "$OUT/pytest_gpu.txt"
fi
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
