#!/bin/bash
# Alternating A/B of library variants built by tools/ablate.sh (GPU box).
#   bash tools/ab.sh TAG "v1 v2 v1 v2" [bench args...]   -> gpurun_out/TAG/ab.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/$1
mkdir -p "$OUT"
: > "$OUT/ab.jsonl"
for v in $2; do
  echo "{\"variant\": \"$v\"}" >> "$OUT/ab.jsonl"
  OM_LIB=$PWD/_abl/lib_$v.so timeout -k 10 200 python bench.py --warmup 1 --no-cpu-baseline --no-extras "${@:3}" \
      >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err" || { echo "variant $v failed"; exit 1; }
done
echo ok
