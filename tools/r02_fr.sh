set -o pipefail
OUT=gpurun_out/r02_fr
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $OUT/pytest_gpu.txt 2>&1 || { echo pytest failed; exit 1; }
STEPS=16 VARIANTS="base nofastrej base nofastrej" timeout -k 10 600 bash tools/ablate.sh run r02_fr || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/serial -o run --output-format csv -- python bench.py --no-cpu-baseline --streams 1 --steps 4 --warmup 1 > $OUT/serial.json 2> $OUT/serial.err || { echo serial failed; exit 1; }
timeout -k 10 300 python tools/path_census.py 480 270 16 > $OUT/census.txt 2>&1 || { echo census failed; exit 1; }
echo ok
