#!/bin/bash
# r04 late: the C1_adaptive bench entry, then tail-threshold re-sweeps on the current kernels
# (C3 with half-precision nodes, C4, C1), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_q4; mkdir -p $OUT
timeout -k 10 300 python -c "import bench,types,json; a=types.SimpleNamespace(streams=2,kernel='auto',pipeline='auto'); print(json.dumps(bench.run_adaptive(a)))" > $OUT/c1_adaptive.json || exit 1
cat $OUT/c1_adaptive.json
bash tools/sweep.sh r04_q4 "C3 T8|--config C3 --tail 8" "C3 T10|--config C3 --tail 10" "C3 T12|--config C3 --tail 12" "C3 T14|--config C3 --tail 14" \
  "C3 T8|--config C3 --tail 8" "C3 T10|--config C3 --tail 10" "C3 T12|--config C3 --tail 12" "C3 T14|--config C3 --tail 14" \
  "C4 T20|--config C4 --steps 4 --tail 20" "C4 T24|--config C4 --steps 4 --tail 24" "C4 T32|--config C4 --steps 4 --tail 32" \
  "C4 T20|--config C4 --steps 4 --tail 20" "C4 T24|--config C4 --steps 4 --tail 24" "C4 T32|--config C4 --steps 4 --tail 32" \
  "C1 T14|--tail 14" "C1 T16|--tail 16" "C1 T20|--tail 20" "C1 T14|--tail 14" "C1 T16|--tail 16" "C1 T20|--tail 20" || exit 1
echo ok
