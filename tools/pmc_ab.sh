#!/bin/bash
# One SQ counter pass per library variant (tools/ablate.sh builds) over a short C1 bench run.
#   [PMC="counters (at most 8 SQ_)"] bash tools/pmc_ab.sh TAG "v1 v2 ..." [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p "$OUT"
for v in $2; do
  OM_LIB=$PWD/_abl/lib_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc ${PMC:-SQ_INSTS_VALU SQ_ACTIVE_INST_VALU \
      SQ_INSTS_VALU_TRANS_F32 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_SALU SQ_WAIT_INST_ANY} \
      -d "$OUT/$v" -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-extras "${@:3}" \
      > "$OUT/$v.log" 2>&1 || { echo "pmc $v failed"; exit 1; }
done
echo ok
