"""Per-launch durations of one timed bench step from a rocprofv3 kernel trace.
Usage: python tools/trace_step.py gpurun_out/TAG/prof/run_kernel_trace.csv [step_index]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else 3
starts = [i for i, r in enumerate(rows) if "k_bounce<" in r["Kernel_Name"] and ", false, false, true>" in r["Kernel_Name"]]
i0 = starts[min(k, len(starts) - 1)]
tot = 0.0
out = []
for r in rows[i0:]:
    name = r["Kernel_Name"].split("(")[0].split("::")[-1]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    gap = 0.0
    tot += d
    out.append(f"{name}:{d:.0f}")
    if "k_accumulate" in name:
        break
span = (int(rows[i0 + len(out) - 1]["End_Timestamp"]) - int(rows[i0]["Start_Timestamp"])) / 1e3
print(" ".join(out))
print(f"launches {len(out)} busy {tot:.0f} us span {span:.0f} us")
