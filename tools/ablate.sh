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
# Variants of the current sources.  The code variants that measured slower in r01-r03 were
# deleted in r04 (their numbers stay in DESIGN.md §5/§8 and git history); what is left is the
# exactness ablations (timing only: results differ from the oracle) and the tunables of
# raytracingoneweekend_amd/csrc/om_tuning.h (bit-identical results).
declare -A V=(
  [base]="$COMMON $DEV"
  [fastdiv]="$COMMON --offload-arch=gfx950 -fno-hip-fp32-correctly-rounded-divide-sqrt -fno-gpu-flush-denormals-to-zero -fno-slp-vectorize"
  [contract]="${COMMON/-ffp-contract=off/-ffp-contract=fast} $DEV"
  [ftz]="$COMMON --offload-arch=gfx950 -fhip-fp32-correctly-rounded-divide-sqrt -fgpu-flush-denormals-to-zero -fno-slp-vectorize"
  # workgroup size x waves-per-SIMD request
  [b256w8]="$COMMON $DEV -DOM_WF_BLOCK=256 -DOM_WF_WAVES=8"
  [b1024w8]="$COMMON $DEV -DOM_WF_BLOCK=1024 -DOM_WF_WAVES=8"
  [b512w6]="$COMMON $DEV -DOM_WF_BLOCK=512 -DOM_WF_WAVES=6"
  [tspb1]="$COMMON $DEV -DOM_WF_TAIL_SPB=1"
  [tspb4]="$COMMON $DEV -DOM_WF_TAIL_SPB=4"
  # segments per CU (lanes per CU / workgroup size), traced and wide (marched, L2 BVH2)
  [lpc2k]="$COMMON $DEV -DOM_WF_LANES_PER_CU=2048"
  [lpc8k]="$COMMON $DEV -DOM_WF_LANES_PER_CU=8192"
  [mlpc4k]="$COMMON $DEV -DOM_WF_LANES_PER_CU_WIDE=4096"
  [mlpc16k]="$COMMON $DEV -DOM_WF_LANES_PER_CU_WIDE=16384"
  # S-10k: bytes of breadth-first BVH2 prefix staged in LDS (0 = all nodes through L2)
  [hyb0]="$COMMON $DEV -DOM_WF_HYB_BYTES=0"
  [hyb16k]="$COMMON $DEV -DOM_WF_HYB_BYTES=16384"
  [hyb40k]="$COMMON $DEV -DOM_WF_HYB_BYTES=40960"
  [hyb28k]="$COMMON $DEV -DOM_WF_HYB_BYTES=28672"
  [hyb8k]="$COMMON $DEV -DOM_WF_HYB_BYTES=8192"
  [hyb12k]="$COMMON $DEV -DOM_WF_HYB_BYTES=12288"
  [hyb20k]="$COMMON $DEV -DOM_WF_HYB_BYTES=20480"
  # S-10k with --kernel bvh4: bytes of breadth-first half-precision BVH4 prefix in LDS (default 0)
  [h4p8k]="$COMMON $DEV -DOM_WF_HYB4_BYTES=8192"
  [h4p4k]="$COMMON $DEV -DOM_WF_HYB4_BYTES=4096"
  [h4p12k]="$COMMON $DEV -DOM_WF_HYB4_BYTES=12288"
  # k_march: refill threshold, steps per refill check
  [refill8]="$COMMON $DEV -DOM_WF_REFILL=8"
  [refill24]="$COMMON $DEV -DOM_WF_REFILL=24"
  # marched tail: ended lanes shaded together once this many wait
  [tm0]="$COMMON $DEV -DOM_WF_TAIL_MARCHED=0"
  [tm0l16]="$COMMON $DEV -DOM_WF_TAIL_MARCHED=0 -DOM_WF_LANES_PER_CU_WIDE=16384"
  [tmw7]="$COMMON $DEV -DOM_WF_TAIL_MARCH_WAVES=7"
  [tmw6]="$COMMON $DEV -DOM_WF_TAIL_MARCH_WAVES=6"
  [tsh1]="$COMMON $DEV -DOM_WF_TAIL_SHADE=1"
  [tsh4]="$COMMON $DEV -DOM_WF_TAIL_SHADE=4"
  [tsh8]="$COMMON $DEV -DOM_WF_TAIL_SHADE=8"
  [tsh16]="$COMMON $DEV -DOM_WF_TAIL_SHADE=16"
  [tsh32]="$COMMON $DEV -DOM_WF_TAIL_SHADE=32"
  [tmu4]="$COMMON $DEV -DOM_WF_TAIL_UNROLL=4"
  [tmu12]="$COMMON $DEV -DOM_WF_TAIL_UNROLL=12"
  [tmu16]="$COMMON $DEV -DOM_WF_TAIL_UNROLL=16"
  [tmu24]="$COMMON $DEV -DOM_WF_TAIL_UNROLL=24"
  [tmu32]="$COMMON $DEV -DOM_WF_TAIL_UNROLL=32"
  [tmu16mu12]="$COMMON $DEV -DOM_WF_TAIL_UNROLL=16 -DOM_MARCH_UNROLL=12"
  [tmu16mu16]="$COMMON $DEV -DOM_WF_TAIL_UNROLL=16 -DOM_MARCH_UNROLL=16"
  [trf8]="$COMMON $DEV -DOM_WF_TAIL_REFILL=8"
  [trf32]="$COMMON $DEV -DOM_WF_TAIL_REFILL=32"
  [mu4]="$COMMON $DEV -DOM_MARCH_UNROLL=4"
  [mu12]="$COMMON $DEV -DOM_MARCH_UNROLL=12"
  # adaptive wavefront: tail threshold of adaptive batches
  [adt16]="$COMMON $DEV -DOM_WF_ADAPTIVE_TAIL=16"
  # batch shape: 2^25 paths for every frame (C4 in 4-spp batches), 8 / 32-spp batches
  [mp25]="$COMMON $DEV -DOM_WF_MAX_PATHS_LOG2=25"
  [bs8]="$COMMON $DEV -DOM_WF_BATCH_SPP=8 -DOM_WF_MIN_PATHS_LOG2=20"
  [bs32]="$COMMON $DEV -DOM_WF_BATCH_SPP=32"
  [mn24]="$COMMON $DEV -DOM_WF_MIN_PATHS_LOG2=24"
  [mn26]="$COMMON $DEV -DOM_WF_MIN_PATHS_LOG2=26"
  # k_accumulate: loads of 1 / 4 / 16 samples issued together
  [acc1]="$COMMON $DEV -DOM_ACC_GROUP=1"
  [acc4]="$COMMON $DEV -DOM_ACC_GROUP=4"
  [acc16]="$COMMON $DEV -DOM_ACC_GROUP=16"
  # BVH builder: max SAH leaf size, traversal cost (host side, om_bvh.cpp)
  [bl2]="$COMMON $DEV -DOM_BVH_MAX_LEAF=2"
  [bl4]="$COMMON $DEV -DOM_BVH_MAX_LEAF=4"
  [bl1]="$COMMON $DEV -DOM_BVH_MAX_LEAF=1 -DOM_BVH_LEAF_FORCE=1"
  [bl3]="$COMMON $DEV -DOM_BVH_MAX_LEAF=3"
  [bl2t05]="$COMMON $DEV -DOM_BVH_MAX_LEAF=2 -DOM_BVH_TRAV=0.5"
  [bt05]="$COMMON $DEV -DOM_BVH_TRAV=0.5"
  [bt2]="$COMMON $DEV -DOM_BVH_TRAV=2.0"
  # r06: BVH2 f32 LDS node stride (bank slots; default 80)
  [p64]="$COMMON $DEV -DOM_B2_NODE_STRIDE=64"
  [p96]="$COMMON $DEV -DOM_B2_NODE_STRIDE=96"
  [p112]="$COMMON $DEV -DOM_B2_NODE_STRIDE=112"
  # LLVM AMDGPU scheduler strategies (same code, different instruction order)
  [ilp]="$COMMON $DEV -mllvm -amdgpu-sched-strategy=max-ilp"
  [memclause]="$COMMON $DEV -mllvm -amdgpu-sched-strategy=max-memory-clause"
)
if [ "$1" = list ]; then echo "${!V[@]}"; exit 0; fi
if [ "$1" = resources ]; then
  for k in ${VARIANTS:-${!V[@]}}; do
    echo "== $k"; /opt/rocm/bin/hipcc ${V[$k]} -c -x hip $SRC/om_wavefront.hip -o /dev/null -Rpass-analysis=kernel-resource-usage 2>&1 | \
      grep -E "Function Name|VGPRs:|ScratchSize|Occupancy" | sed -E 's/.*remark: +//; s/ \[-Rpass.*//' | paste - - - - | \
      grep -E "k_(bounce|tail)ILi6ELb0ELb0" | awk '{print substr($3,1,40), $5, $8, $11}'
  done
  exit 0
fi
if [ "$1" = build ]; then
  mkdir -p _abl
  for k in ${VARIANTS:-${!V[@]}}; do
    ( printf 'extern "C" const char* om_build_id(void) { return "ablate-%s"; }\n' "$k" > _abl/bid_$k.cpp && \
      /opt/rocm/bin/hipcc ${V[$k]} -shared -o _abl/lib_$k.so $SRC/om_world.cpp $SRC/om_bvh.cpp $SRC/om_image.cpp $SRC/om_tiles.cpp \
        $SRC/om_shard.cpp _abl/bid_$k.cpp -x hip $SRC/om_render.hip $SRC/om_wavefront.hip $SRC/om_display.hip $SRC/om_multi.hip \
        -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib > _abl/$k.log 2>&1 && echo "built $k" ) &
  done
  wait
  exit 0
fi
TAG=${2:-abl}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
: > "$OUT/abl.jsonl"
for k in ${VARIANTS:-base fastdiv contract ftz}; do
  echo "{\"variant\": \"$k\"}" >> "$OUT/abl.jsonl"
  OM_LIB=$PWD/_abl/lib_$k.so timeout -k 10 200 python bench.py --steps ${STEPS:-8} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} "${@:3}" \
      >> "$OUT/abl.jsonl" 2>> "$OUT/abl.err" || { echo "variant $k failed"; exit 1; }
done
echo ok
