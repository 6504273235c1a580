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
  # scheduling variants (bit-identical results): workgroup size x waves-per-SIMD request (0 = none)
  [b256]="$COMMON $DEV -DOM_WF_BLOCK=256 -DOM_WF_WAVES=0"
  [b256w8]="$COMMON $DEV -DOM_WF_BLOCK=256 -DOM_WF_WAVES=8"
  [b512]="$COMMON $DEV -DOM_WF_BLOCK=512 -DOM_WF_WAVES=0"
  [b1024w8]="$COMMON $DEV -DOM_WF_BLOCK=1024 -DOM_WF_WAVES=8"
  # cost split of the fused bounce kernel: run one half twice
  [trace2x]="$COMMON $DEV -DOM_ABLATE_TRACE2X"
  [tspb1]="$COMMON $DEV -DOM_WF_TAIL_SPB=1"
  [tspb4]="$COMMON $DEV -DOM_WF_TAIL_SPB=4"
  [shade2x]="$COMMON $DEV -DOM_ABLATE_SHADE2X"
  [b512w6]="$COMMON $DEV -DOM_WF_BLOCK=512 -DOM_WF_WAVES=6"
  # bounce work distribution (bit-identical): block-step scan instead of per-wave LDS queues,
  # unaligned segments, both (the r01_v6 kernel)
  [waveq0]="$COMMON $DEV -DOM_WF_WAVEQ=0"
  [align1]="$COMMON $DEV -DOM_WF_ALIGN=1"
  [v6]="$COMMON $DEV -DOM_WF_WAVEQ=0 -DOM_WF_ALIGN=1"
  # segments per CU (lanes per CU / workgroup size)
  [b1024l8]="$COMMON $DEV -DOM_WF_BLOCK=1024 -DOM_WF_WAVES=8 -DOM_WF_LANES_PER_CU=8192"
  # correctly rounded 1/d for the slab tests (the default uses the hardware reciprocal)
  [invdiv]="$COMMON $DEV -DOM_EXACT_INVDIR"
  # S-10k: bytes of breadth-first BVH2 prefix staged in LDS (0 = all nodes through L2)
  [hyb0]="$COMMON $DEV -DOM_WF_HYB_BYTES=0"
  [hyb16k]="$COMMON $DEV -DOM_WF_HYB_BYTES=16384"
  [hyb40k]="$COMMON $DEV -DOM_WF_HYB_BYTES=40960"
  # marched worlds: the fused trace+march+shade bounce kernel instead of k_march + shade
  [msplit0]="$COMMON $DEV -DOM_WF_MARCH_SPLIT=0"
  [marrays]="$COMMON $DEV -DOM_MARCH_ARRAYS_ONLY"
  [mregs1]="$COMMON $DEV -DOM_WF_MARCH_REGS=1"
  [refill12]="$COMMON $DEV -DOM_WF_REFILL=12"
  [refill24]="$COMMON $DEV -DOM_WF_REFILL=24"
  [refill8]="$COMMON $DEV -DOM_WF_REFILL=8"
  [refill16]="$COMMON $DEV -DOM_WF_REFILL=16"
  [refill48]="$COMMON $DEV -DOM_WF_REFILL=48"
  [refill64]="$COMMON $DEV -DOM_WF_REFILL=64"
  # adaptive wavefront: samples per pixel per serial batch
  [ab1]="$COMMON $DEV -DOM_WF_ADAPTIVE_BATCH=1"
  [ab4]="$COMMON $DEV -DOM_WF_ADAPTIVE_BATCH=4"
  [ab16]="$COMMON $DEV -DOM_WF_ADAPTIVE_BATCH=16"
  # slab-test the unbounded always2 records too (the default skips their box)
  [infslab]="$COMMON $DEV -DOM_ALWAYS2_INF_SLAB"
  [late]="$COMMON $DEV -DOM_WF_EARLY_REST=0"
  [lpc2k]="$COMMON $DEV -DOM_WF_LANES_PER_CU=2048"
  [lpc8k]="$COMMON $DEV -DOM_WF_LANES_PER_CU=8192"
  [lpc16k]="$COMMON $DEV -DOM_WF_LANES_PER_CU=16384"
  # r02: lanes per CU for marched worlds and L2-resident BVH2s (default 8192)
  [mlpc4k]="$COMMON $DEV -DOM_WF_LANES_PER_CU_WIDE=4096"
  [mlpc16k]="$COMMON $DEV -DOM_WF_LANES_PER_CU_WIDE=16384"
  [w6k]="$COMMON $DEV -DOM_WF_LANES_PER_CU_WIDE=6144"
  [w12k]="$COMMON $DEV -DOM_WF_LANES_PER_CU_WIDE=12288"
  # r02: bounce 0's occupancy request (waves per SIMD; default = OM_WF_WAVES)
  [first7]="$COMMON $DEV -DOM_WF_WAVES_FIRST=7"
  [first6]="$COMMON $DEV -DOM_WF_WAVES_FIRST=6"
  [lpc6k]="$COMMON $DEV -DOM_WF_LANES_PER_CU=6144"
  [lpc3k]="$COMMON $DEV -DOM_WF_LANES_PER_CU=3072"
  # r02: Sphere::hit without the divisions when both roots are provably rejected (default off:
  # -0.4% on C1 over two A/B pairs at 32 and 128 spp per call, profiles/r02_v3)
  [fastrej]="$COMMON $DEV -DOM_SPHERE_FAST_REJECT=1"
  [nofastrej]="$COMMON $DEV -DOM_SPHERE_FAST_REJECT=0"
  # r02: async tails (each batch's tail + accumulate on a high-priority tail stream)
  [async]="$COMMON $DEV -DOM_WF_ASYNC_TAIL=1"
  [aspb4]="$COMMON $DEV -DOM_WF_ASYNC_TAIL=1 -DOM_WF_TAIL_SPB_ASYNC=4"
  [aspb8]="$COMMON $DEV -DOM_WF_ASYNC_TAIL=1 -DOM_WF_TAIL_SPB_ASYNC=8"
  # r02: the axis-aligned ground sphere's diagonal test (default on); packed slab FMAs on the
  # interleaved BVH2 node layout
  [nodiag]="$COMMON $DEV -DOM_DIAG_SPHERE=0"
  [pkslab]="$COMMON $DEV -DOM_PK_SLAB=1"
  [pkslabl]="$COMMON $DEV -DOM_PK_SLAB=1 -DOM_WF_EARLY_REST=0"
  # r03: march escape test (default off: C2 -35% march steps, time neutral, profiles/r02_v8)
  [noesc]="$COMMON $DEV -DOM_MARCH_ESCAPE=0"
  [esc]="$COMMON $DEV -DOM_MARCH_ESCAPE=1"
  # r02: software-pipelined marched-object loads in the march step (default off: C2 -7%)
  [pf]="$COMMON $DEV -DOM_MARCH_PREFETCH=1"
  [escregs]="$COMMON $DEV -DOM_MARCH_ESCAPE=1 -DOM_WF_MARCH_REGS=1"
  # r03: marched-only worlds trace with the scratch-stack BVH instead of the reference loop
  [bvhfb]="$COMMON $DEV -DOM_EMPTY_B2_BRUTE=0"
  # r02: LLVM AMDGPU scheduler strategies (same code, different instruction order)
  [ilp]="$COMMON $DEV -mllvm -amdgpu-sched-strategy=max-ilp"
  [memclause]="$COMMON $DEV -mllvm -amdgpu-sched-strategy=max-memory-clause"
  [bias0]="$COMMON $DEV -mllvm -amdgpu-schedule-metric-bias=0"
  [tprio0]="$COMMON $DEV -DOM_WF_ASYNC_TAIL=1 -DOM_WF_TAIL_PRIO=0"
  # r03: async drain: a batch's bounces >= K, tail and accumulate on its tail stream (4 queue sets)
  [drain4]="$COMMON $DEV -DOM_WF_ASYNC_TAIL=1 -DOM_WF_TAIL_PRIO=0 -DOM_WF_DRAIN_AT=4"
  [drain6]="$COMMON $DEV -DOM_WF_ASYNC_TAIL=1 -DOM_WF_TAIL_PRIO=0 -DOM_WF_DRAIN_AT=6"
  [drain8]="$COMMON $DEV -DOM_WF_ASYNC_TAIL=1 -DOM_WF_TAIL_PRIO=0 -DOM_WF_DRAIN_AT=8"
  [drain6p]="$COMMON $DEV -DOM_WF_ASYNC_TAIL=1 -DOM_WF_TAIL_PRIO=1 -DOM_WF_DRAIN_AT=6"
  # r03: C2's k_march with the SDF-only exact register view (default on) or the arrays view
  [noexact]="$COMMON $DEV -DOM_WF_MARCH_EXACT=0"
  [exactlds]="$COMMON $DEV -DOM_WF_MARCH_EXACT=2"
  [exactsgpr]="$COMMON $DEV -DOM_WF_MARCH_EXACT=1"
  # r03: diagnostic build, per-phase wave cycles (tools/phase_stamps.py)
  [phase]="$COMMON $DEV -DOM_PHASE_STAMPS=1"
  [phase2]="$COMMON $DEV -DOM_PHASE_STAMPS=2"
  # r03: BVH2 stack top in a register (the pop's LDS read off the critical path)
  [tos]="$COMMON $DEV -DOM_B2_TOS=1"
  # r03: always2 records through scalar loads (default on) or vector loads
  [a2vec]="$COMMON $DEV -DOM_A2_SCALAR=0"
  # r03: two paths per lane in the later bounces (k_bounce2), occupancy request 0 (none) / 6 / 5
  [dual]="$COMMON $DEV -DOM_WF_DUAL=1 -DOM_B2_DIRECT=0"
  # r03: bounce 0's tile lists through vector loads only (default: scalar when the wave is one tile)
  [tilesvec]="$COMMON $DEV -DOM_TILES_UNIFORM=0"
  # r03: one rand_in_unit_sphere loop for Lambertian and Metal lanes (default) or one per kind
  [scat2]="$COMMON $DEV -DOM_SCATTER_SHARED_SPHERE=0"
  # r03: leaf codes through the leaf table (default: direct first/count codes when they fit)
  [leaftab]="$COMMON $DEV -DOM_B2_DIRECT=0"
  # r03: 2^25 paths per batch (r02) instead of 2^27: C4's 4K frame in 4-spp batches
  [mp25]="$COMMON $DEV -DOM_WF_MAX_PATHS_LOG2=25"
  # r03: bounce 0's tile-list sphere tests with the division-free rejection (default on)
  [tfr0]="$COMMON $DEV -DOM_TILES_FAST_REJECT=0"
  # r03: bounce 0's depth-sorted tile lists without the wave early-out
  [teo0]="$COMMON $DEV -DOM_TILES_EARLY_OUT=0"
  # r03: bounce 0's tile candidates: sphere pairs interleaved (measured -0.4%, default off)
  [tpair1]="$COMMON $DEV -DOM_TILES_PAIRED=1"
  # r02 knob, run at last: bounce 0's occupancy request 7 / 6 waves per SIMD (default 8)
  [first7b]="$COMMON $DEV -DOM_WF_WAVES_FIRST=7"
  [dual6]="$COMMON $DEV -DOM_WF_DUAL=1 -DOM_WF_DUAL_WAVES=6 -DOM_B2_DIRECT=0"
  [dual5]="$COMMON $DEV -DOM_WF_DUAL=1 -DOM_WF_DUAL_WAVES=5 -DOM_B2_DIRECT=0"
  # r03: merged late bounces (from bounce M, F segments per workgroup) and grouped accumulate loads
  [m6f4]="$COMMON $DEV -DOM_WF_MERGE_AT=6 -DOM_WF_MERGE=4"
  [m8f4]="$COMMON $DEV -DOM_WF_MERGE_AT=8 -DOM_WF_MERGE=4"
  [m6f8]="$COMMON $DEV -DOM_WF_MERGE_AT=6 -DOM_WF_MERGE=8"
  [m10f8]="$COMMON $DEV -DOM_WF_MERGE_AT=10 -DOM_WF_MERGE=8"
  [acc8]="$COMMON $DEV -DOM_ACC_GROUP=8"
  [acc1]="$COMMON $DEV -DOM_ACC_GROUP=1"
  [acc8m8f4]="$COMMON $DEV -DOM_ACC_GROUP=8 -DOM_WF_MERGE_AT=8 -DOM_WF_MERGE=4"
  # r03: accumulates on their own stream (no lockstep through the accumulate chain), with and
  # without a stagger of stream 1's first batch, with merged late bounces
  [as]="$COMMON $DEV -DOM_ACC_GROUP=8 -DOM_WF_ACC_STREAM=1"
  [asm]="$COMMON $DEV -DOM_ACC_GROUP=8 -DOM_WF_ACC_STREAM=1 -DOM_WF_MERGE_AT=8 -DOM_WF_MERGE=4"
  [asmst4]="$COMMON $DEV -DOM_ACC_GROUP=8 -DOM_WF_ACC_STREAM=1 -DOM_WF_MERGE_AT=8 -DOM_WF_MERGE=4 -DOM_WF_STAGGER=4"
  [asst4]="$COMMON $DEV -DOM_ACC_GROUP=8 -DOM_WF_ACC_STREAM=1 -DOM_WF_STAGGER=4"
  [asst2]="$COMMON $DEV -DOM_ACC_GROUP=8 -DOM_WF_ACC_STREAM=1 -DOM_WF_STAGGER=2"
  # r03: late bounces read the BVH2 through the caches (no LDS staging) from bounce K
  [lg6]="$COMMON $DEV -DOM_ACC_GROUP=8 -DOM_WF_LATE_GLOBAL=6"
  [lg9]="$COMMON $DEV -DOM_ACC_GROUP=8 -DOM_WF_LATE_GLOBAL=9"
  [lg12]="$COMMON $DEV -DOM_ACC_GROUP=8 -DOM_WF_LATE_GLOBAL=12"
  # r03: march SDF roots as hipcc's sqrt core when the whole wave is in range (same bits)
  [sqcore]="$COMMON $DEV -DOM_MARCH_SQRT_CORE=1"
  [sqall]="$COMMON $DEV -DOM_SQRT_CORE=1"
  # r03: the always2 records loaded up front (unrolled, <= 4 records)
  [a2p]="$COMMON $DEV -DOM_A2_PRELOAD=1"
  # r03: non-temporal hints on the path-state loads / stores (component loads, same registers)
  [ntl]="$COMMON $DEV -DOM_WF_NT_LOADS=1 -DOM_WF_NT_STORES=0"
  [nt0]="$COMMON $DEV -DOM_WF_NT_LOADS=0 -DOM_WF_NT_STORES=0"
  [nts]="$COMMON $DEV -DOM_WF_NT_LOADS=0 -DOM_WF_NT_STORES=1"
  [ntls]="$COMMON $DEV -DOM_WF_NT_LOADS=1 -DOM_WF_NT_STORES=1"
  # r03: 32-spp batches (2^26 paths at 1080p) instead of 16
  [bs32]="$COMMON $DEV -DOM_WF_BATCH_SPP=32"
  # r03: k_march steps per refill check
  [mu2]="$COMMON $DEV -DOM_MARCH_UNROLL=2"
  [mu4]="$COMMON $DEV -DOM_MARCH_UNROLL=4"
  [mu2r8]="$COMMON $DEV -DOM_MARCH_UNROLL=2 -DOM_WF_REFILL=8"
  [mu8]="$COMMON $DEV -DOM_MARCH_UNROLL=8"
  [mu6]="$COMMON $DEV -DOM_MARCH_UNROLL=6"
  [mu4r24]="$COMMON $DEV -DOM_MARCH_UNROLL=4 -DOM_WF_REFILL=24"
  [mu4r32]="$COMMON $DEV -DOM_MARCH_UNROLL=4 -DOM_WF_REFILL=32"
  [mu8r32]="$COMMON $DEV -DOM_MARCH_UNROLL=8 -DOM_WF_REFILL=32"
  [mu1]="$COMMON $DEV -DOM_MARCH_UNROLL=1"
  # r03: raised wave priority for the tail / the accumulate (s_setprio)
  [tp2]="$COMMON $DEV -DOM_WF_TAIL_SETPRIO=2"
  [tp3]="$COMMON $DEV -DOM_WF_TAIL_SETPRIO=3"
  [tpa2]="$COMMON $DEV -DOM_WF_TAIL_SETPRIO=2 -DOM_ACC_SETPRIO=2"
  [mu12]="$COMMON $DEV -DOM_MARCH_UNROLL=12"
  [mu16]="$COMMON $DEV -DOM_MARCH_UNROLL=16"
  [mu8r12]="$COMMON $DEV -DOM_MARCH_UNROLL=8 -DOM_WF_REFILL=12"
  [bs8]="$COMMON $DEV -DOM_WF_BATCH_SPP=8 -DOM_WF_MIN_PATHS_LOG2=20"
  [bs12]="$COMMON $DEV -DOM_WF_BATCH_SPP=12 -DOM_WF_MIN_PATHS_LOG2=20"
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
for k in ${VARIANTS:-base fastdiv contract rng32 ftz}; do
  echo "{\"variant\": \"$k\"}" >> "$OUT/abl.jsonl"
  OM_LIB=$PWD/_abl/lib_$k.so timeout -k 10 200 python bench.py --steps ${STEPS:-8} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} "${@:3}" \
      >> "$OUT/abl.jsonl" 2>> "$OUT/abl.err" || { echo "variant $k failed"; exit 1; }
done
echo ok
