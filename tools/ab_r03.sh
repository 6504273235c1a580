#!/bin/bash
# Round-3 A/B experiments on the GPU box, one per name (the variants are tools/ablate.sh builds in
# _abl/; build them first with `VARIANTS="..." bash tools/ablate.sh build`).  Each run checks the
# candidate build's parity through OM_LIB where it changes code, then alternates the variants.
#   bash tools/ab_r03.sh EXPERIMENT [TAG]      -> gpurun_out/TAG/...
# EXPERIMENT: kernel_c3 | merge | accstream | lateglobal | sqcore | nt | batch | batch2 | munroll | munroll2 | munroll3 | setprio | sqall | a2p | tailC2 | tailC2b | tailC3 | tailC3b | tailC4 | tailC4b
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
EXP=$1
TAG=${2:-r03_$EXP}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
parity() {   # variant, test files...
  local v=$1; shift
  OM_LIB=$PWD/_abl/lib_$v.so timeout -k 10 400 python -u -m pytest "$@" -m gpu -x -q --timeout 200 --timeout-method thread \
      -p no:cacheprovider > "$OUT/pytest_$v.txt" 2>&1 || { echo "pytest $v failed"; return 1; }
  tail -1 "$OUT/pytest_$v.txt"
}
bench_runs() {   # file, then "label|args" items
  local f=$OUT/$1; shift
  : > "$f"
  for item in "$@"; do
    echo "{\"variant\": \"${item%%|*}\"}" >> "$f"
    timeout -k 10 200 python bench.py --warmup 1 --no-cpu-baseline --no-extras ${item#*|} >> "$f" 2>> "$OUT/bench.err" || return 1
  done
}
P="tests/test_gpu_parity.py tests/test_gpu_edge_cases.py"
case $EXP in
  kernel_c3)    # BVH4 vs BVH2 on C3 (L2-resident tree) and C1; C2's tail threshold
    bench_runs ab_bvh4_C3_C1.jsonl "C3 auto|--config C3" "C3 bvh4|--config C3 --kernel bvh4" "C3 auto|--config C3" \
        "C3 bvh4|--config C3 --kernel bvh4" "C1 auto|" "C1 bvh4|--kernel bvh4" || exit 1
    bench_runs tail_sweep_C2.jsonl "C2 tail 16|--config C2 --tail 16" "C2 tail 24|--config C2 --tail 24" \
        "C2 tail 32|--config C2 --tail 32" "C2 tail 16|--config C2 --tail 16" "C2 tail 24|--config C2 --tail 24" \
        "C2 tail 32|--config C2 --tail 32" || exit 1 ;;
  merge)        # merged late bounces, grouped accumulate loads
    parity m6f8 $P || exit 1; parity acc8m8f4 $P || exit 1
    bash tools/ab.sh "$TAG/ab_merge" "base m8f4 m6f4 m6f8 m10f8 acc8 acc8m8f4 acc8m8f4 acc8 m10f8 m6f8 m6f4 m8f4 base" || exit 1 ;;
  accstream)    # accumulate stream, stagger
    parity asst4 $P tests/test_multi_gpu.py || exit 1
    bash tools/ab.sh "$TAG/ab_accstream" "acc8 as asst2 asst4 asmst4 asmst4 asst4 asst2 as acc8" || exit 1 ;;
  lateglobal)   # late bounces through the caches
    parity lg6 $P || exit 1
    bash tools/ab.sh "$TAG/ab_lateglobal" "base lg6 lg9 lg12 lg12 lg9 lg6 base" || exit 1 ;;
  sqcore)       # bare sqrt core in the march SDFs (C2)
    parity sqcore $P || exit 1
    bash tools/ab.sh "$TAG/ab_sqcore_C2" "base sqcore sqcore base base sqcore" --config C2 || exit 1 ;;
  nt)           # non-temporal path-state loads / stores
    parity ntls $P || exit 1
    bash tools/ab.sh "$TAG/ab_nt" "nt0 ntl nts ntls ntls nts ntl nt0" || exit 1 ;;
  batch)        # 32-spp batches; 3 and 4 streams
    bash tools/ab.sh "$TAG/ab_bs32_128" "base bs32 bs32 base" || exit 1
    bash tools/ab.sh "$TAG/ab_bs32_256" "base bs32 bs32 base" --spp-per-step 256 --steps 2 || exit 1
    bench_runs streams.jsonl "streams 2 spp/call 128|--streams 2 --spp-per-step 128 --steps 4" \
        "streams 3 spp/call 96|--streams 3 --spp-per-step 96 --steps 6" "streams 3 spp/call 192|--streams 3 --spp-per-step 192 --steps 3" \
        "streams 4 spp/call 128|--streams 4 --spp-per-step 128 --steps 4" "streams 2 spp/call 128|--streams 2 --spp-per-step 128 --steps 4" \
        "streams 3 spp/call 96|--streams 3 --spp-per-step 96 --steps 6" "streams 3 spp/call 192|--streams 3 --spp-per-step 192 --steps 3" \
        "streams 4 spp/call 128|--streams 4 --spp-per-step 128 --steps 4" || exit 1 ;;
  batch2)       # 8- and 12-spp batches
    bash tools/ab.sh "$TAG/ab_bs8_128" "base bs8 bs8 base" || exit 1
    bash tools/ab.sh "$TAG/ab_bs12_96" "base bs12 bs12 base" --spp-per-step 96 --steps 6 || exit 1 ;;
  munroll)      # k_march steps per refill check (C2)
    parity mu2 $P || exit 1
    bash tools/ab.sh "$TAG/ab_munroll_C2" "base mu2 mu4 mu2r8 mu2r8 mu4 mu2 base" --config C2 || exit 1 ;;
  munroll2)     # more steps per check, refill thresholds (C2)
    parity mu8 $P || exit 1
    bash tools/ab.sh "$TAG/ab_munroll2_C2" "mu4 mu6 mu8 mu4r24 mu4r32 mu8r32 mu8r32 mu4r32 mu4r24 mu8 mu6 mu4" --config C2 || exit 1 ;;
  munroll3)     # around the default (8 steps per check)
    bash tools/ab.sh "$TAG/ab_munroll3_C2" "base mu12 mu16 mu8r12 mu8r12 mu16 mu12 base" --config C2 || exit 1 ;;
  setprio)      # raised wave priority for the tail / accumulate (C1, then C2)
    bash tools/ab.sh "$TAG/ab_setprio_C1" "base tp2 tp3 tpa2 tpa2 tp3 tp2 base" || exit 1
    bash tools/ab.sh "$TAG/ab_setprio_C2" "base tp2 tp2 base" --config C2 || exit 1 ;;
  sqall)        # the bare sqrt core in unit() and the sphere tests (C1, C3)
    parity sqall $P || exit 1
    bash tools/ab.sh "$TAG/ab_sqall_C1" "base sqall sqall base base sqall" || exit 1
    bash tools/ab.sh "$TAG/ab_sqall_C3" "base sqall sqall base" --config C3 || exit 1 ;;
  a2p)          # the always2 records loaded up front (C1, C3)
    parity a2p $P || exit 1
    bash tools/ab.sh "$TAG/ab_a2p_C1" "base a2p a2p base base a2p" || exit 1
    bash tools/ab.sh "$TAG/ab_a2p_C3" "base a2p a2p base" --config C3 || exit 1 ;;
  tailC2)       # C2's tail threshold on the 8-steps-per-check k_march
    bench_runs tail_sweep_C2.jsonl "C2 tail 12|--config C2 --tail 12" "C2 tail 16|--config C2 --tail 16" \
        "C2 tail 20|--config C2 --tail 20" "C2 tail 24|--config C2 --tail 24" "C2 tail 24|--config C2 --tail 24" \
        "C2 tail 20|--config C2 --tail 20" "C2 tail 16|--config C2 --tail 16" "C2 tail 12|--config C2 --tail 12" || exit 1 ;;
  tailC2b)      # lower tail thresholds on C2
    bench_runs tail_sweep_C2b.jsonl "C2 tail 6|--config C2 --tail 6" "C2 tail 8|--config C2 --tail 8" \
        "C2 tail 10|--config C2 --tail 10" "C2 tail 12|--config C2 --tail 12" "C2 tail 16|--config C2 --tail 16" \
        "C2 tail 16|--config C2 --tail 16" "C2 tail 12|--config C2 --tail 12" "C2 tail 10|--config C2 --tail 10" \
        "C2 tail 8|--config C2 --tail 8" "C2 tail 6|--config C2 --tail 6" || exit 1 ;;
  tailC3)       # C3's tail threshold (BVH2 through L2)
    bench_runs tail_sweep_C3.jsonl "C3 tail 12|--config C3 --tail 12" "C3 tail 16|--config C3 --tail 16" \
        "C3 tail 20|--config C3 --tail 20" "C3 tail 20|--config C3 --tail 20" "C3 tail 16|--config C3 --tail 16" \
        "C3 tail 12|--config C3 --tail 12" || exit 1 ;;
  tailC3b)      # lower tail thresholds on C3
    bench_runs tail_sweep_C3b.jsonl "C3 tail 6|--config C3 --tail 6" "C3 tail 8|--config C3 --tail 8" \
        "C3 tail 10|--config C3 --tail 10" "C3 tail 12|--config C3 --tail 12" "C3 tail 12|--config C3 --tail 12" \
        "C3 tail 10|--config C3 --tail 10" "C3 tail 8|--config C3 --tail 8" "C3 tail 6|--config C3 --tail 6" || exit 1 ;;
  tailC4)       # C4's tail threshold (4K frame, 16-spp batches of 133M paths)
    bench_runs tail_sweep_C4.jsonl "C4 tail 12|--config C4 --tail 12" "C4 tail 16|--config C4 --tail 16" \
        "C4 tail 20|--config C4 --tail 20" "C4 tail 24|--config C4 --tail 24" "C4 tail 24|--config C4 --tail 24" \
        "C4 tail 20|--config C4 --tail 20" "C4 tail 16|--config C4 --tail 16" "C4 tail 12|--config C4 --tail 12" || exit 1 ;;
  tailC4b)      # higher tail thresholds on C4
    bench_runs tail_sweep_C4b.jsonl "C4 tail 24|--config C4 --tail 24" "C4 tail 28|--config C4 --tail 28" \
        "C4 tail 32|--config C4 --tail 32" "C4 tail 32|--config C4 --tail 32" "C4 tail 28|--config C4 --tail 28" \
        "C4 tail 24|--config C4 --tail 24" || exit 1 ;;
  *) echo "unknown experiment $EXP"; exit 2 ;;
esac
echo ok
