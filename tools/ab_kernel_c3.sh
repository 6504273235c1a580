set -o pipefail
cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/${TAG:-r03_v9}
mkdir -p $OUT
: > $OUT/ab_c3_bvh4.jsonl
for v in auto bvh4 auto bvh4; do
  echo "{\"variant\": \"C3 $v\"}" >> $OUT/ab_c3_bvh4.jsonl
  timeout -k 10 200 python bench.py --config C3 --kernel $v --warmup 1 --no-cpu-baseline --no-extras >> $OUT/ab_c3_bvh4.jsonl 2>> $OUT/ab.err || exit 1
done
for v in auto bvh4; do
  echo "{\"variant\": \"C1 $v\"}" >> $OUT/ab_c3_bvh4.jsonl
  timeout -k 10 200 python bench.py --config C1 --kernel $v --warmup 1 --no-cpu-baseline --no-extras >> $OUT/ab_c3_bvh4.jsonl 2>> $OUT/ab.err || exit 1
done
echo ok1
# C2: tail threshold re-check on the r03 tree (the tail runs at ~4% lane utilisation on C2)
: > gpurun_out/r03_v9/tail_sweep_C2.jsonl
for t in 16 24 32 16 24 32; do
  echo "{\"variant\": \"C2 tail $t\"}" >> gpurun_out/r03_v9/tail_sweep_C2.jsonl
  timeout -k 10 200 python bench.py --config C2 --tail $t --warmup 1 --no-cpu-baseline --no-extras >> gpurun_out/r03_v9/tail_sweep_C2.jsonl 2>> gpurun_out/r03_v9/ab.err || exit 1
done
echo ok2
