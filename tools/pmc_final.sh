#!/bin/bash
# End-of-round PMC passes (GPU box), summarised on the box so gpurun_out/ stays small:
#   C1 all five passes -> pmc_summary_C1.json + pmc_traffic.json; C2 all five -> *_C2.json;
#   C3 all five -> *_C3.json; C4 all five -> *_C4.json; C1_adaptive (the bench's adaptive frame,
#   tools/adaptive_bench.py, concurrent schedule only) all five -> *_C1_adaptive.json.
#   Raw pass files are deleted.
#   [CONFIGS="C1 C2 C3 C4"] bash tools/pmc_final.sh TAG      -> gpurun_out/TAG/pmc_*.json
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-pmc_final}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
run() {   # name, passes, bench args...
  local name=$1 passes=$2; shift 2
  PASSES="$passes" bash tools/pmc.sh "$TAG/raw_$name" "$@" > "$OUT/pmc_$name.log" 2>&1 || { echo "pmc $name failed"; return 1; }
  if [ "$passes" != "3 4" ]; then
    python tools/pmc_summary.py "$OUT/raw_$name" > "$OUT/pmc_summary_$name.json" || return 1
  fi
  python tools/pmc_traffic.py "$OUT/raw_$name" "$OUT/pmc_traffic_$name.json" || return 1
  rm -rf "$OUT/raw_$name"
}
case " ${CONFIGS:-C1 C2 C3 C4 C1_adaptive} " in *" C1 "*) run C1 "1 2 3 4 5" --no-extras || exit 1 ;; esac
case " ${CONFIGS:-C1 C2 C3 C4 C1_adaptive} " in *" C2 "*) run C2 "1 2 3 4 5" --config C2 --no-extras || exit 1 ;; esac
case " ${CONFIGS:-C1 C2 C3 C4 C1_adaptive} " in *" C3 "*) run C3 "1 2 3 4 5" --config C3 --no-extras || exit 1 ;; esac
case " ${CONFIGS:-C1 C2 C3 C4 C1_adaptive} " in *" C4 "*) run C4 "1 2 3 4 5" --config C4 --no-extras || exit 1 ;; esac
case " ${CONFIGS:-C1 C2 C3 C4 C1_adaptive} " in *" C1_adaptive "*)
  export AD_NO_SERIAL=1 AD_NO_MEGA=1 PMC_CMD="python tools/adaptive_bench.py 128 C1 512"
  run C1_adaptive "1 2 3 4 5" || exit 1; unset PMC_CMD ;; esac
echo ok
