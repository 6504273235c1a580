#!/bin/bash
# r04 late: fused k_march_shade for marched worlds' bounce 0 -- parity (marched GPU tests + the
# bench's oracle window on the ms1 build), then the C2 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04_q9; mkdir -p $OUT
OM_LIB=$PWD/_abl/lib_ms1.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "marched or torus or auto_pipeline or production or kitchen" > $OUT/pytest_ms1.txt 2>&1 || { tail -30 $OUT/pytest_ms1.txt; exit 1; }
tail -1 $OUT/pytest_ms1.txt
OM_LIB=$PWD/_abl/lib_ms1.so timeout -k 10 300 python bench.py --config C2 --no-cpu-baseline > $OUT/bench_ms1_C2.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench_ms1_C2.json').read().strip().splitlines()[-1]); print(d['value'], d['window_parity'])"
NO_TESTS=1 bash tools/ab_quick.sh r04_q9 "base ms1 ms1u16 ms1u24 base ms1 ms1u16 ms1u24" "C2" || exit 1
echo ok
