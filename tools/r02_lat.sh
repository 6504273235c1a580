#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02_lat
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/lone50 -o run --output-format csv -- python tools/lone_latency.py > $OUT/lone50.txt 2>&1 || { echo lone50 failed; exit 1; }
LL_TAIL=1 timeout -k 10 120 rocprofv3 --kernel-trace -d $OUT/lone1 -o run --output-format csv -- python tools/lone_latency.py > $OUT/lone1.txt 2>&1 || { echo lone1 failed; exit 1; }
bash tools/r02_async.sh r02_lat "32" "base nofastrej base nofastrej" || exit 1
echo ok
