#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02_streams; mkdir -p $OUT; : > $OUT/sweep.jsonl
for C in C2 C3; do for S in 2 4 1 2 4; do
  timeout -k 10 200 python bench.py --config $C --streams $S --warmup 1 --no-cpu-baseline --no-extras >> $OUT/sweep.jsonl 2>> $OUT/sweep.err || { echo "fail $C $S"; exit 1; }
done; done
echo ok
