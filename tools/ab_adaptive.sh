#!/bin/bash
# GPU box: tools/adaptive_bench.py per library build (_abl/lib_<v>.so), alternating.
#   bash tools/ab_adaptive.sh TAG "v1 v2 v1 v2" [STEP] [SCENE] [SPP]   -> gpurun_out/TAG/adaptive.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; VARS=$2; STEP=${3:-64}; SCENE=${4:-C1}; SPP=${5:-64}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for v in $VARS; do
  echo "{\"variant\": \"$v\"}" >> "$OUT/adaptive.jsonl"
  OM_LIB=$PWD/_abl/lib_$v.so timeout -k 10 300 python tools/adaptive_bench.py $STEP $SCENE $SPP >> "$OUT/adaptive.jsonl" 2>> "$OUT/ad.err" \
      || { echo "variant $v failed"; exit 1; }
done
echo ok
