#!/bin/bash
# GPU box: rocprofv3 kernel traces of library variants (_abl/lib_<v>.so) on one config, for
# per-kernel timelines (tools/trace_step.py).
#   bash tools/trace_ab.sh TAG "v1 v2" CFG [bench args...]   -> gpurun_out/TAG/<v>/...kernel_trace.csv
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=$1; VARS=$2; CFG=$3; shift 3
mkdir -p gpurun_out/$TAG
for v in $VARS; do
  OM_LIB=$PWD/_abl/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/$v -o run --output-format csv -- \
      python3 bench.py --config $CFG --warmup 1 --no-cpu-baseline --no-window-parity "$@" > gpurun_out/$TAG/$v.log 2>&1 \
      || { echo "trace $v failed"; tail -20 gpurun_out/$TAG/$v.log; exit 1; }
done
echo ok
