"""Summarise rocprofv3 --pmc passes (tools/pmc.sh) for the render kernel.

Usage: python tools/pmc_summary.py gpurun_out/TAG [kernel-substring]
Prints per-dispatch averages of every counter for dispatches whose name contains
the substring (default: the production build `, false>`), plus derived metrics.
HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reads 1/2 of wide
streaming reads on gfx950 -> reported raw and x2; WRITE_SIZE as is.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(tag_dir, sub):
    vals = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(tag_dir, "p*", "*counter_collection.csv"))):
        per = defaultdict(float)
        for row in csv.DictReader(open(f)):
            if sub not in row["Kernel_Name"]:
                continue
            per[(row["Dispatch_Id"], row["Counter_Name"])] += float(row["Counter_Value"])
        agg = defaultdict(list)
        for (d, c), v in per.items():
            agg[c].append(v)
        for c, v in agg.items():
            vals[c] = v
    return {c: sum(v) / len(v) for c, v in vals.items() if v}, {c: len(v) for c, v in vals.items()}


def main():
    tag = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ", false>"
    avg, n = load(tag, sub)
    out = {"kernel_filter": sub, "dispatches": max(n.values()) if n else 0, "counters": avg}
    d = {}
    if "SQ_THREAD_CYCLES_VALU" in avg and "SQ_ACTIVE_INST_VALU" in avg:
        d["valu_lane_utilisation"] = avg["SQ_THREAD_CYCLES_VALU"] / (64.0 * avg["SQ_ACTIVE_INST_VALU"])
    if "SQ_INSTS_VALU" in avg and "SQ_WAVES" in avg:
        d["valu_insts_per_wave"] = avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"]
    if "SQ_WAIT_INST_ANY" in avg and "SQ_WAVE_CYCLES" in avg:
        d["wait_inst_frac"] = avg["SQ_WAIT_INST_ANY"] / avg["SQ_WAVE_CYCLES"]
        d["wait_any_frac"] = avg.get("SQ_WAIT_ANY", 0) / avg["SQ_WAVE_CYCLES"]
        d["active_any_frac"] = avg.get("SQ_ACTIVE_INST_ANY", 0) / avg["SQ_WAVE_CYCLES"]
    if "FETCH_SIZE" in avg:
        d["fetch_bytes_raw"] = avg["FETCH_SIZE"] * 1024
        d["fetch_bytes_x2"] = avg["FETCH_SIZE"] * 2048
    if "WRITE_SIZE" in avg:
        d["write_bytes"] = avg["WRITE_SIZE"] * 1024
    if "fetch_bytes_x2" in d and "write_bytes" in d:
        d["hbm_bytes_per_dispatch_corrected"] = d["fetch_bytes_x2"] + d["write_bytes"]
    out["derived"] = d
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
