#!/bin/bash
# Development check on the GPU box: the -m gpu tests (optionally a -k filter) and one bench line.
#   bash tools/gpu_quick.sh TAG [pytest -k expr] [bench args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-quick}; K=${2:-}; shift 2 2>/dev/null
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ${K:+-k "$K"} \
    > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest failed"; tail -30 "$OUT/pytest_gpu.txt"; exit 1; }
tail -2 "$OUT/pytest_gpu.txt"
timeout -k 10 400 python bench.py "$@" > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail -20 "$OUT/bench.err"; exit 1; }
echo ok
