"""Print the (variant, value, ms/step, march steps/segment) rows of a tools/ab_run.sh / tools/sweep.sh result file."""
import json
import sys

for path in sys.argv[1:]:
    v = None
    for line in open(path):
        if not line.startswith("{"):
            continue
        d = json.loads(line)
        if "variant" in d:
            v = d["variant"]
            continue
        w = d.get("work", {})
        print(f"{path.split('/')[-1]:16s} {v:10s} {d['value']:9.1f} {d['ms_per_step']:8.3f} ms  "
              f"march/seg {w.get('march_steps_per_segment', 0):6.2f}  launch {d['roofline']['avg_launch_ms']:.4f}")
