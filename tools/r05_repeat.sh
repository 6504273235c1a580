#!/bin/bash
# GPU box: the driver's bench shape (--steps 20 --warmup 5) N times on one box, for the run-to-run
# spread of the C1 number (--no-cpu-baseline: the line has no `configs` block).      bash tools/r05_repeat.sh TAG [N]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05_rep}
mkdir -p "$OUT"
: > "$OUT/driver_shape.jsonl"
for i in $(seq 1 "${2:-3}"); do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline >> "$OUT/driver_shape.jsonl" 2>> "$OUT/err.txt" \
      || { echo "bench run $i failed"; exit 1; }
  echo "run $i done"
done
python - "$OUT/driver_shape.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["value"], d["roofline"]["frac"], {k: v["value"] for k, v in (d.get("configs") or {}).items() if v})
PY
