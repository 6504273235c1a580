#!/bin/bash
# GPU box: rocprofv3 kernel trace + stats of the C2 / C3 / C4 bench configs (per-kernel time of
# each config's frame), summaries only.        bash tools/r05_cfgprof.sh TAG
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05_cfgprof}
mkdir -p "$OUT"
for c in C2 C3 C4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$c" -o run --output-format csv -- \
      python bench.py --config $c --no-cpu-baseline --no-extras > "$OUT/bench_$c.json" 2> "$OUT/bench_$c.err" \
      || { echo "rocprof $c failed"; exit 1; }
  S=$(find "$OUT/prof_$c" -name '*kernel_stats.csv' | head -1)
  cp "$S" "$OUT/kernel_stats_$c.csv" && rm -rf "$OUT/prof_$c"
  echo "$c done"
done
echo ok
