#!/bin/bash
# r05 GPU check: full -m gpu suite, smoke, the default bench line; then an optional A/B
# (AB_VARS on AB_CFGS via tools/ab_quick.sh, no tests).  Every step time-limited; stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05_check}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -1 "$OUT/pytest_gpu.txt"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; cat "$OUT/smoke.log"; exit 1; }
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 400 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
fi
if [ -n "$AB_VARS" ]; then
  NO_TESTS=1 bash tools/ab_quick.sh "$TAG/ab" "$AB_VARS" "$AB_CFGS" || exit 1
fi
echo ok
