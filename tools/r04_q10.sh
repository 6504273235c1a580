#!/bin/bash
# r04 late: the L2-resident BVH2's leaf table staged in LDS (OM_WF_L2_LEAVES_LDS) -- S-10k parity on
# the lt12 build, then the C3 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_q10; mkdir -p $OUT
OM_LIB=$PWD/_abl/lib_lt12.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "ten_k or c3_shape" > $OUT/pytest_lt12.txt 2>&1 || { tail -30 $OUT/pytest_lt12.txt; exit 1; }
tail -1 $OUT/pytest_lt12.txt
NO_TESTS=1 bash tools/ab_quick.sh r04_q10 "base lt16 lt12 lt8 base lt16 lt12 lt8" "C3" || exit 1
echo ok
