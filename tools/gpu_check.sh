#!/bin/bash
# GPU-box check used during development (run through gpurun):
#   tests (-m gpu), smoke, bench (N=1), rocprofv3 kernel-trace/stats of the bench.
# Every GPU step has its own time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-dev}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_gpu.txt" 2>&1 || { echo "pytest failed"; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; exit 1; }
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --no-extras > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" || { echo "rocprof failed"; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --kernel-timing launch > "$OUT/bench_launch_timing.json" 2>> "$OUT/bench.err" || { echo "bench (launch timing) failed"; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --kernel-timing off > "$OUT/bench_notiming.json" 2>> "$OUT/bench.err" || { echo "bench (no timing) failed"; exit 1; }
if [ -z "$NO_PMC" ]; then
  CONFIGS=C1 bash tools/pmc_final.sh "$TAG/pmc" > "$OUT/pmc.log" 2>&1 || { echo "pmc failed"; exit 1; }
fi
echo ok
