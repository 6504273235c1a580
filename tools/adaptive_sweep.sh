set -o pipefail
OUT=gpurun_out/s3y; mkdir -p $OUT; : > $OUT/ad.jsonl
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for k in base ab1 ab4 ab16; do
  echo "{\"variant\": \"$k\"}" >> $OUT/ad.jsonl
  OM_LIB=$PWD/_abl/lib_$k.so timeout -k 10 200 python tools/adaptive_bench.py >> $OUT/ad.jsonl 2>> $OUT/ad.err || exit 1
done
echo ok
