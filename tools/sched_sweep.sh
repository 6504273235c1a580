#!/bin/bash
# Wavefront schedule sweep (C1, timing off).  Each argument after TAG is one case:
#   "label|ENV=V ENV2=V|bench args"      e.g. "s2|ENV=1|--streams 2 --spp-per-step 32"
# (The environment knobs of the r01_v6 schedule experiments, OM_WF_BATCHES / OM_WF_STAGGER,
# lived only in experiment builds; the shipped schedule is set through bench.py's --streams,
# --spp-per-step and --tail)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for c in "$@"; do
  IFS='|' read -r label envs args <<< "$c"
  env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --kernel-timing off $args \
      > "$OUT/$label.json" 2> "$OUT/$label.err" || { echo "bench $label failed"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" \
      "$OUT/$label.json" "$label"
done
