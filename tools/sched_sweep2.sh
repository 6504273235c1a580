set -o pipefail
OUT=gpurun_out/s3e; mkdir -p $OUT; : > $OUT/sweep.jsonl
run() { echo "{\"args\": \"$*\"}" >> $OUT/sweep.jsonl; timeout -k 10 200 python bench.py --no-cpu-baseline --kernel-timing off --warmup 1 "$@" >> $OUT/sweep.jsonl 2>> $OUT/sweep.err || exit 1; }
run --steps 16
run --steps 16 --tail 12
run --steps 16 --tail 20
run --steps 16 --tail 24
run --steps 8 --spp-per-step 64 --streams 2
run --steps 8 --spp-per-step 64 --streams 4
run --steps 10 --spp-per-step 48 --streams 3
run --steps 16 --spp-per-step 16 --streams 2
run --steps 16
echo ok
