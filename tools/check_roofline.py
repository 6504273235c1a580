"""Cross-check bench.py's live roofline against rocprofv3 output of the same command.

1. --stats summary: the average duration of the bounce-kernel family (production build) must
   agree with roofline.avg_launch_ms.
2. (optional) --kernel-trace timestamps: per render call (launches between two k_snapshot), the
   family's summed launch durations over the call's span give the launch concurrency, and the
   family's flops (the line's flop_per_launch) over the calls' spans give the chip-level rate and
   `frac` again, independently of bench.py's HIP events.

    python tools/check_roofline.py STATS.csv BENCH.json [KERNEL_TRACE.csv[.gz]]
"""
import csv
import gzip
import json
import re
import sys

FAMILY = re.compile(r"k_(bounce|tail|march)<\d+, false|k_raygen<false>")   # bench.py's bounce family


def trace_check(path, bench):
    f = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
    rows = sorted(csv.DictReader(f), key=lambda r: int(r["Start_Timestamp"]))
    calls, cur = [], None
    for r in rows:
        name = r["Kernel_Name"]
        if "k_snapshot" in name:
            cur = []
            calls.append(cur)
        elif cur is not None and FAMILY.search(name):
            cur.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    calls = [c for c in calls if c]
    # the timed calls and the per-launch rerun both run the production build; keep the calls
    # with the line's launch count per step
    per_step = round(bench["roofline"]["launches_per_step"])
    calls = [c for c in calls if len(c) == per_step]
    busy = sum(e - s for c in calls for s, e in c)
    span = sum(max(e for _, e in c) - min(s for s, _ in c) for c in calls)
    launches = sum(len(c) for c in calls)
    r = bench["roofline"]
    eff_ms = span / launches / 1e6
    achieved = r["flop_per_launch"] / (eff_ms / 1e3) / 1e12
    return {"trace_calls": len(calls), "trace_launches": launches,
            "trace_launch_concurrency": round(busy / span, 3), "bench_launch_concurrency": r["launch_concurrency"],
            "trace_effective_ms_per_launch": round(eff_ms, 4), "bench_effective_ms_per_launch": r["effective_ms_per_launch"],
            "trace_achieved_tflops": round(achieved, 3), "trace_frac": round(achieved / r["peak"], 4),
            "bench_frac": r["frac"], "frac_ratio": round(r["frac"] / (achieved / r["peak"]), 4)}


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if FAMILY.search(r["Name"])]
    calls = sum(int(r["Calls"]) for r in rows)
    total_ns = sum(float(r["TotalDurationNs"]) for r in rows)
    bench = json.loads([l for l in open(sys.argv[2]).read().splitlines() if l.startswith("{")][-1])
    live = bench["roofline"]["avg_launch_ms"]
    prof = total_ns / calls / 1e6
    out = {"rocprof_family_calls": calls, "rocprof_avg_launch_ms": round(prof, 4), "bench_avg_launch_ms": live,
           "ratio": round(live / prof, 4),
           "per_kernel": {re.search(r"k_\w+<[^>]*>", r["Name"]).group(0): {"calls": int(r["Calls"]),
                                                                            "avg_us": round(float(r["AverageNs"]) / 1e3, 1)}
                          for r in rows}}
    if len(sys.argv) > 3:
        out.update(trace_check(sys.argv[3], bench))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
