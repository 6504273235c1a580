#!/bin/bash
# Overlapped-schedule sweep (C1, timing off): batches per call x stagger bounce.
#   bash tools/overlap_sweep.sh TAG "B1 B2 ..." "S1 S2 ..." [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-overlap}; BS=${2:-"0 2 4"}; SS=${3:-"2 3 4"}; shift 3
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for b in $BS; do
  for s in $SS; do
    [ "$b" -lt 2 ] && [ "$s" != "$(echo $SS | cut -d' ' -f1)" ] && continue
    OM_WF_BATCHES=$b OM_WF_STAGGER=$s timeout -k 10 200 python bench.py --no-cpu-baseline --kernel-timing off "$@" \
        > "$OUT/b${b}_s${s}.json" 2> "$OUT/b${b}_s${s}.err" || { echo "bench b=$b s=$s failed"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'])" \
        "$OUT/b${b}_s${s}.json" $b $s
  done
done
