#!/bin/bash
# async-tail A/B over samples per call (GPU box).  Usage: bash tools/r02_async.sh TAG "spp list" "variants" [pytest]
set -o pipefail
OUT=gpurun_out/${1:-r02_async}
SPPS=${2:-"32 128 512"}
VARS=${3:-"base noasync base noasync"}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$4" ]; then
  OM_LIB=$PWD/_abl/lib_async.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "concurrent or progressive or adaptive or shallow" > $OUT/pytest_async.txt 2>&1 || { echo async pytest failed; exit 1; }
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo pytest failed; exit 1; }
fi
: > $OUT/sweep.jsonl
for spp in $SPPS; do
  steps=$((1024 / spp))
  for v in $VARS; do
    echo "{\"variant\": \"$v\", \"spp\": $spp}" >> $OUT/sweep.jsonl
    OM_LIB=$PWD/_abl/lib_$v.so timeout -k 10 200 python bench.py --steps $steps --warmup 1 --spp-per-step $spp --no-cpu-baseline --no-extras >> $OUT/sweep.jsonl 2>> $OUT/sweep.err || { echo "bench $v $spp failed"; exit 1; }
  done
done
if [ -n "$TRACE" ]; then
  OM_LIB=$PWD/_abl/lib_$TRACE.so timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/trace -o run --output-format csv -- python bench.py --no-cpu-baseline --steps 2 --warmup 1 --spp-per-step 128 > $OUT/trace.json 2> $OUT/trace.err || { echo trace failed; exit 1; }
fi
echo ok
