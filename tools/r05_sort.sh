#!/bin/bash
# GPU box: survivor ordering by (origin cell, octant) key (_abl/lib_sort.so) and AoS path records
# alone (_abl/lib_aos.so) vs the default build: parity of both through OM_LIB, then C1/C4 A/B.
# The two variants were built from commit 17acef0 (tools/ablate.sh sort / aos there); both lost
# and the code was removed after it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r05_sort}
mkdir -p "$OUT" _abl
cp raytracingoneweekend_amd/libottomarcher.so _abl/lib_base.so
for v in sort aos; do
  OM_LIB=$PWD/_abl/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
      --timeout 120 --timeout-method thread -p no:cacheprovider > "$OUT/pytest_$v.txt" 2>&1 \
      || { echo "pytest $v failed"; tail -30 "$OUT/pytest_$v.txt"; exit 1; }
  tail -1 "$OUT/pytest_$v.txt"
done
for c in C1 C4; do
  : > "$OUT/ab_$c.jsonl"
  for v in base sort aos base sort aos; do
    echo "{\"variant\": \"$v\"}" >> "$OUT/ab_$c.jsonl"
    OM_LIB=$PWD/_abl/lib_$v.so timeout -k 10 200 python bench.py --config $c --warmup 2 --no-cpu-baseline --no-window-parity \
        >> "$OUT/ab_$c.jsonl" 2>> "$OUT/ab.err" || { echo "variant $v $c failed"; exit 1; }
  done
done
python tools/ab_print.py "$OUT"/ab_*.jsonl
echo ok
