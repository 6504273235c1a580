#!/bin/bash
# End-of-round evidence, part 2: the bench at the driver's shape, then the PMC passes (C1-C4).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:-final}
mkdir -p gpurun_out/$TAG
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/$TAG/bench_driver.json 2> gpurun_out/$TAG/bench_driver.err || { echo "bench failed"; exit 1; }
bash tools/pmc_final.sh "${TAG}_pmc" || { echo "pmc failed"; exit 1; }
echo ok
