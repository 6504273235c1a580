#!/bin/bash
# End-of-round evidence in one GPU call: tests, smoke, bench + rocprofv3 (gpu_check.sh), the PMC passes of
# every config, then the bench line again with those PMC summaries in place (matches_timed_build).
#   bash tools/final_evidence.sh   -> gpurun_out/r06_final6/, gpurun_out/r06_final6_pmc/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
NO_PMC=1 bash tools/gpu_check.sh r06_final6 || exit 1
bash tools/pmc_final.sh r06_final6_pmc > gpurun_out/r06_final6/pmc_final.log 2>&1 || { echo pmc failed; exit 1; }
P=gpurun_out/r06_final6_pmc
for c in C1 C2 C3 C4 C1_adaptive; do cp $P/pmc_summary_$c.json profiles/; done
cp $P/pmc_traffic_C1.json profiles/pmc_traffic.json
for c in C2 C3 C4 C1_adaptive; do cp $P/pmc_traffic_$c.json profiles/; done
timeout -k 10 300 python bench.py > gpurun_out/r06_final6/bench_final.json 2> gpurun_out/r06_final6/bench_final.err || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06_final6/driver1.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/r06_final6/driver2.json 2>/dev/null || exit 1
echo ok
