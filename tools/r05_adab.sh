#!/bin/bash
# r05: adaptive A/B of library builds (_abl/lib_<v>.so) on C1 adaptive, alternating, with the
# runtime schedules of $SCHEDS; then (PROF=1) a kernel trace of the first variant.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05_adab}; VARS=${2:-"base"}
mkdir -p "$OUT"
: > "$OUT/ab.jsonl"
for v in $VARS; do
  echo "{\"variant\": \"$v\"}" >> "$OUT/ab.jsonl"
  OM_LIB=$PWD/_abl/lib_$v.so AD_TAIL=${AD_TAIL:-0} AD_NO_MEGA=1 AD_NO_SERIAL=1 AD_SCHEDS="${SCHEDS:-3,23}" \
      timeout -k 10 300 python tools/adaptive_bench.py 128 C1 512 >> "$OUT/ab.jsonl" 2>> "$OUT/err.txt" || { echo "variant $v failed"; exit 1; }
done
python3 - "$OUT/ab.jsonl" <<'PY'
import json, sys
var = None
for line in open(sys.argv[1]):
    d = json.loads(line)
    if "variant" in d: var = d["variant"]; continue
    for k, v in d.items():
        if isinstance(v, dict): print(f"{var:8s} {k:22s} {v['s']*1e3:6.1f} ms taken {v['taken_msamples_s']:7.1f} seg {v['segments_g']:.3f} G {v['gseg_s']:.2f} G/s")
PY
if [ -n "$PROF" ]; then
  v=${VARS%% *}
  OM_LIB=$PWD/_abl/lib_$v.so AD_TAIL=${AD_TAIL:-0} AD_NO_MEGA=1 AD_NO_SERIAL=1 AD_SCHEDS="" timeout -k 10 300 \
      rocprofv3 --kernel-trace --output-format csv -d "$OUT/prof" -o run -- python3 tools/adaptive_bench.py 128 C1 512 > "$OUT/prof.json" 2>> "$OUT/err.txt" || exit 1
  gzip -c "$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)" > "$OUT/kernel_trace.csv.gz" && rm -rf "$OUT/prof"
fi
echo ok
