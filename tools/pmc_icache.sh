#!/bin/bash
# Instruction-cache counters over a short C1 bench run (one rocprofv3 --pmc pass, kernel trace only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-pmc_icache}
mkdir -p "$OUT"
timeout -s KILL 60 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || true
grep -o "SQC_[A-Z_]*ICACHE[A-Z_]*\|SQ_IFETCH[A-Z_]*" "$OUT/avail.txt" | sort -u > "$OUT/icache_counters.txt" || true
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE \
    -d "$OUT/p1" -o run --output-format csv -- python bench.py --steps 4 --warmup 1 --no-cpu-baseline --no-extras \
    > "$OUT/p1.log" 2>&1 || { echo "pmc icache pass failed"; exit 1; }
echo ok
