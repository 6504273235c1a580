#!/bin/bash
# Bench every (pipeline, kernel) variant briefly; one JSON line each in gpurun_out/TAG/variants.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-variants}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
: > "$OUT/variants.jsonl"
for PIPE in ${PIPES:-wavefront megakernel}; do
  for K in ${KERNELS:-bvh4 bvh2 sbvh bvh culled}; do
    timeout -k 10 200 python bench.py --steps ${STEPS:-8} --warmup 1 --no-cpu-baseline --pipeline $PIPE --kernel $K "$@" \
        >> "$OUT/variants.jsonl" 2>> "$OUT/variants.err" || { echo "variant $PIPE/$K failed"; exit 1; }
  done
done
echo ok
