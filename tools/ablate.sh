#!/bin/bash
# Timing ablations: build variants of libottomarcher.so that each drop ONE exactness
# constraint (results differ from the oracle — timing only), then bench each.
#   bash tools/ablate.sh build        (here: cross-compiles into _abl/)
#   bash tools/ablate.sh run TAG      (GPU box: one JSON line per variant)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SRC=raytracingoneweekend_amd/csrc
COMMON="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -Wno-unused-function"
DEV="--offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-slp-vectorize"
declare -A V=(
  [base]="$COMMON $DEV"
  [fastdiv]="$COMMON --offload-arch=gfx950 -fno-hip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-slp-vectorize"
  [contract]="${COMMON/-ffp-contract=off/-ffp-contract=fast} $DEV"
  [rng32]="$COMMON $DEV -DOM_ABLATE_RNG"
  [ftz]="$COMMON --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -fgpu-flush-denormals-to-zero -fno-slp-vectorize"
)
if [ "$1" = build ]; then
  mkdir -p _abl
  for k in "${!V[@]}"; do
    ( /opt/rocm/bin/hipcc ${V[$k]} -shared -o _abl/lib_$k.so $SRC/om_world.cpp $SRC/om_bvh.cpp -x hip $SRC/om_render.hip $SRC/om_wavefront.hip \
      > _abl/$k.log 2>&1 && echo "built $k" ) &
  done
  wait
  exit 0
fi
TAG=${2:-abl}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
: > "$OUT/abl.jsonl"
for k in ${VARIANTS:-base fastdiv contract rng32 ftz}; do
  echo "{\"variant\": \"$k\"}" >> "$OUT/abl.jsonl"
  OM_LIB=$PWD/_abl/lib_$k.so timeout -k 10 200 python bench.py --steps 8 --warmup 1 --no-cpu-baseline "${@:3}" \
      >> "$OUT/abl.jsonl" 2>> "$OUT/abl.err" || { echo "variant $k failed"; exit 1; }
done
echo ok
