#!/bin/bash
# r05: adaptive schedule sweep on C1 (512 spp adaptive in 128-spp calls): streams, batches per
# stream, target paths and the tail threshold, all runtime knobs (one build).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r05_ad}
mkdir -p "$OUT"
: > "$OUT/sweep.jsonl"
for t in ${TAILS:-0 8 12}; do
  echo "{\"tail\": $t}" >> "$OUT/sweep.jsonl"
  AD_TAIL=$t AD_NO_MEGA=1 AD_SCHEDS="${SCHEDS:-3,24;6,24;8,23}" timeout -k 10 300 python tools/adaptive_bench.py 128 C1 512 ${STREAMS:-3,4} \
      >> "$OUT/sweep.jsonl" 2>> "$OUT/err.txt" || { echo "tail $t failed"; exit 1; }
done
python3 - "$OUT/sweep.jsonl" <<'PY'
import json, sys
tail = None
for line in open(sys.argv[1]):
    d = json.loads(line)
    if "tail" in d: tail = d["tail"]; continue
    for k, v in d.items():
        if isinstance(v, dict): print(f"tail {tail:2d} {k:22s} {v['s']*1e3:6.1f} ms taken {v['taken_msamples_s']:7.1f} seg {v['segments_g']:.3f} G {v['gseg_s']:.2f} G/s")
    print("bit_identical", d["schedules_bit_identical"])
PY
