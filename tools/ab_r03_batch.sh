#!/bin/bash
# r03: batch size and stream count on C1: 32-spp batches (OM_WF_BATCH_SPP, tools/ablate.sh) at 128 and
# 256 spp per call; 3 streams x 16 spp at 96 and 192 spp per call (runtime flags, default build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r03_v14}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/ab.sh "$TAG/ab_bs32_128" "base bs32 bs32 base" || exit 1
bash tools/ab.sh "$TAG/ab_bs32_256" "base bs32 bs32 base" --spp-per-step 256 --steps 2 || exit 1
: > "$OUT/streams.jsonl"
for a in "2 128 4" "3 96 6" "3 192 3" "4 128 4" "2 128 4" "3 96 6" "3 192 3" "4 128 4"; do
  set -- $a
  echo "{\"variant\": \"streams $1 spp/call $2\"}" >> "$OUT/streams.jsonl"
  timeout -k 10 200 python bench.py --warmup 1 --no-cpu-baseline --no-extras --streams $1 --spp-per-step $2 --steps $3 \
      >> "$OUT/streams.jsonl" 2>> "$OUT/streams.err" || { echo "streams $1 failed"; exit 1; }
done
echo ok
