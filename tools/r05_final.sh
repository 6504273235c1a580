#!/bin/bash
# r05 end-of-round evidence on the GPU box (no tests: tools/r05_check.sh runs them):
#   bench line (default run) and the driver's shape (--steps 20 --warmup 5), rocprofv3 kernel trace
#   + stats of the C1 headline, the launch-timing and no-timing lines, the roofline cross-check,
#   and a rocprofv3 kernel trace + stats of the adaptive frame.  Each step time-limited; the chain
#   stops at the first failure.        bash tools/r05_final.sh TAG  -> gpurun_out/TAG/...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-r05_final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 500 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo "bench failed"; tail "$OUT/bench.err"; exit 1; }
echo "bench done"
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > "$OUT/bench_driver.json" 2>> "$OUT/bench.err" || { echo "bench (driver shape) failed"; exit 1; }
echo "bench driver shape done"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
    python bench.py --no-cpu-baseline --no-extras > "$OUT/bench_prof.json" 2> "$OUT/bench_prof.err" || { echo "rocprof failed"; exit 1; }
echo "rocprof done"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --kernel-timing launch > "$OUT/bench_launch_timing.json" 2>> "$OUT/bench.err" || { echo "bench (launch timing) failed"; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-extras --kernel-timing off > "$OUT/bench_notiming.json" 2>> "$OUT/bench.err" || { echo "bench (no timing) failed"; exit 1; }
S=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -1); T=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -1)
cp "$S" "$OUT/kernel_stats.csv" && gzip -c "$T" > "$OUT/kernel_trace.csv.gz" && rm -rf "$OUT/prof"
python tools/check_roofline.py "$OUT/kernel_stats.csv" "$OUT/bench_prof.json" "$OUT/kernel_trace.csv.gz" > "$OUT/roofline_check.json" || { echo "roofline check failed"; exit 1; }
AD_NO_SERIAL=1 AD_NO_MEGA=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/adprof" -o run --output-format csv -- \
    python tools/adaptive_bench.py 128 C1 512 > "$OUT/adaptive_prof.json" 2> "$OUT/adaptive_prof.err" || { echo "adaptive rocprof failed"; exit 1; }
S=$(find "$OUT/adprof" -name '*kernel_stats.csv' | head -1); T=$(find "$OUT/adprof" -name '*kernel_trace.csv' | head -1)
cp "$S" "$OUT/adaptive_kernel_stats.csv" && gzip -c "$T" > "$OUT/adaptive_kernel_trace.csv.gz" && rm -rf "$OUT/adprof"
echo ok
