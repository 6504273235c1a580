#!/bin/bash
# Sweep the wavefront tail bounce (om_set_tail_bounce); one JSON line each in gpurun_out/TAG/tail.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-tail}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
: > "$OUT/tail.jsonl"
for T in ${TAILS:-2 3 4 5 6 8 10 50}; do
  timeout -k 10 200 python bench.py --steps ${STEPS:-8} --warmup 1 --no-cpu-baseline --tail $T "$@" \
      >> "$OUT/tail.jsonl" 2>> "$OUT/tail.err" || { echo "tail $T failed"; exit 1; }
done
echo ok
