set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04_ad; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.txt 2>&1 || { tail -30 $OUT/pytest_gpu.txt; exit 1; }
tail -1 $OUT/pytest_gpu.txt
for st in 16 64; do for sc in C1 C2; do
  timeout -k 10 300 python tools/adaptive_bench.py $st $sc >> $OUT/adaptive.jsonl 2>> $OUT/ad.err || exit 1
done; done
cat $OUT/adaptive.jsonl
: > $OUT/c2s1.jsonl
for it in "mega|--pipeline megakernel" "wave|--pipeline wavefront" "mega|--pipeline megakernel" "wave|--pipeline wavefront"; do
  echo "{\"variant\": \"${it%%|*}\"}" >> $OUT/c2s1.jsonl
  timeout -k 10 200 python bench.py --config C2 --streams 1 --steps 2 --warmup 1 --no-cpu-baseline --no-window-parity --no-extras ${it#*|} >> $OUT/c2s1.jsonl 2>> $OUT/ad.err || exit 1
done
python tools/ab_print.py $OUT/c2s1.jsonl
echo ok
