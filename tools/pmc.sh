#!/bin/bash
# PMC counter passes (rocprofv3 --pmc, each pass its own run, kernel-trace only —
# never combined with sys/runtime traces) over a short bench run.  Usage:
#   [PASSES="3 4"] bash tools/pmc.sh TAG [bench args...]     (default: all five passes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-pmc}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
ARGS="--steps 4 --warmup 1 --no-cpu-baseline --no-window-parity $*"
# PMC_CMD: another program to profile (e.g. the adaptive frame, tools/adaptive_bench.py)
CMD=${PMC_CMD:-"python bench.py $ARGS"}
# the build the passes profile (om_build_id), for bench.py's pmc fields (pmc_summary.py reads it)
python -c "from raytracingoneweekend_amd import _lib as L; print(L.build_id())" > "$OUT/build_id.txt" || exit 1
i=0
for PASS in "SQ_WAVES SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS" \
            "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FLOPS_FP32 SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_VMEM" \
            "FETCH_SIZE" "WRITE_SIZE" "SQ_IFETCH SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64"; do
  i=$((i+1))
  case " ${PASSES:-1 2 3 4 5} " in *" $i "*) ;; *) continue ;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $PASS -d "$OUT/p$i" -o run --output-format csv -- \
      $CMD > "$OUT/p$i.log" 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
echo ok
