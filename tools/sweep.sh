#!/bin/bash
# GPU box: one bench line per "label|bench args" item, in order (alternate items for an A/B).
#   bash tools/sweep.sh TAG "C2 T8|--config C2 --tail 8" "C2 T12|--config C2 --tail 12" ...
#   -> gpurun_out/TAG/sweep.jsonl ({"variant": label} before each line)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
: > "$OUT/sweep.jsonl"
for item in "$@"; do
  echo "{\"variant\": \"${item%%|*}\"}" >> "$OUT/sweep.jsonl"
  timeout -k 10 200 python bench.py --warmup 2 --no-cpu-baseline --no-window-parity --no-extras ${item#*|} \
      >> "$OUT/sweep.jsonl" 2>> "$OUT/sweep.err" || { echo "item $item failed"; exit 1; }
done
python tools/ab_print.py "$OUT/sweep.jsonl"
echo ok
