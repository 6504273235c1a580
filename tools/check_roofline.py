"""Cross-check bench.py's live roofline against the rocprofv3 --stats summary of the same
command: the average duration of the bounce-kernel family (production build) must agree
with roofline.avg_launch_ms.

    python tools/check_roofline.py gpurun_out/TAG/prof/run_kernel_stats.csv gpurun_out/TAG/bench_prof.json
"""
import csv
import json
import re
import sys

FAMILY = re.compile(r"k_(bounce|tail|march)<\d+, false|k_raygen<false>")   # bench.py's bounce family

rows = [r for r in csv.DictReader(open(sys.argv[1])) if FAMILY.search(r["Name"])]
calls = sum(int(r["Calls"]) for r in rows)
total_ns = sum(float(r["TotalDurationNs"]) for r in rows)
bench = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
live = bench["roofline"]["avg_launch_ms"]
prof = total_ns / calls / 1e6
out = {"rocprof_family_calls": calls, "rocprof_avg_launch_ms": round(prof, 4), "bench_avg_launch_ms": live,
       "ratio": round(live / prof, 4), "per_kernel": {re.search(r"k_\w+<[^>]*>", r["Name"]).group(0): {"calls": int(r["Calls"]),
                                                                          "avg_us": round(float(r["AverageNs"]) / 1e3, 1)}
                                                      for r in rows}}
print(json.dumps(out, indent=1))
