"""Per-dispatch SQ counters of the bounce-kernel family for each variant of tools/pmc_ab.sh."""
import collections
import csv
import glob
import os
import sys

for d in sorted(glob.glob(os.path.join(sys.argv[1], "*", ""))):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not f:
        continue
    agg = collections.defaultdict(float)
    disp = set()
    for r in csv.DictReader(open(f[0])):
        k = r["Kernel_Name"]
        if "k_bounce" in k or "k_tail" in k:
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp.add(r["Dispatch_Id"])
    n = max(len(disp), 1)
    print(os.path.basename(d.rstrip("/")), "dispatches", n,
          " ".join(f"{c}={v / n / 1e6:.2f}M" for c, v in sorted(agg.items())))
