"""Summarise rocprofv3 --pmc passes (tools/pmc.sh), per kernel.

Usage: python tools/pmc_summary.py gpurun_out/TAG [kernel-regex]

Every dispatch of every pass file is read; a counter's value for a dispatch is the sum of its
rows (rocprofv3 writes one row per counter and dispatch, or per XCD/SE instance).  Dispatches
are grouped by kernel name (the name up to its argument list), and the groups whose name
matches the regex (default: the production bounce family) are reported with, per
counter, the mean over that kernel's dispatches AND the number of dispatches it was measured on
(each pass is its own run, so counters come from different dispatches of the same kernels).
`combined` is the dispatch-weighted mean over the matching kernels, counter by counter.
HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reads 1/2 of wide streaming reads
on gfx950 -> reported raw and x2; WRITE_SIZE as is.
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


# the production (COUNT = false) bounce family: the kernels bench.py's roofline covers
PRODUCTION_FAMILY = r"^(k_(bounce|tail|march)<\d+, false|k_raygen<false>)"


def kernel_key(name):
    """`void ns::k_bounce<6, false, false, false, false>(OmSceneDev, ...)` -> `k_bounce<6, false, false, false, false>`"""
    name = name.replace("(anonymous namespace)::", "").split("(")[0]
    name = re.sub(r"^void\s+", "", name)
    return re.sub(r"^.*::(?=k_|render_kernel)", "", name)


def load(tag_dir):
    """-> {kernel: {counter: [value per dispatch]}}"""
    per = defaultdict(float)
    kname = {}
    for f in sorted(glob.glob(os.path.join(tag_dir, "p*", "*counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            key = (f, row["Dispatch_Id"])
            kname[key] = kernel_key(row["Kernel_Name"])
            per[(key, row["Counter_Name"])] += float(row["Counter_Value"])
    out = defaultdict(lambda: defaultdict(list))
    for (key, counter), v in per.items():
        out[kname[key]][counter].append(v)
    return out


def derived(avg):
    d = {}
    if "SQ_THREAD_CYCLES_VALU" in avg and "SQ_ACTIVE_INST_VALU" in avg:
        d["valu_lane_utilisation"] = avg["SQ_THREAD_CYCLES_VALU"] / (64.0 * avg["SQ_ACTIVE_INST_VALU"])
    if "SQ_INSTS_VALU" in avg and "SQ_WAVES" in avg:
        d["valu_insts_per_wave"] = avg["SQ_INSTS_VALU"] / avg["SQ_WAVES"]
    if "SQ_INSTS_SALU" in avg and "SQ_INSTS_VALU" in avg:
        d["salu_per_valu"] = avg["SQ_INSTS_SALU"] / avg["SQ_INSTS_VALU"]
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
    return d


def summarise(tag, pattern):
    data = load(tag)
    rx = re.compile(pattern)
    kernels, tot, cnt = {}, defaultdict(float), defaultdict(int)
    for k in sorted(data):
        if not rx.search(k):
            continue
        avg = {c: sum(v) / len(v) for c, v in data[k].items()}
        kernels[k] = {"dispatches": {c: len(v) for c, v in data[k].items()}, "counters": avg, "derived": derived(avg)}
        for c, v in data[k].items():
            tot[c] += sum(v)
            cnt[c] += len(v)
    comb = {c: tot[c] / cnt[c] for c in tot}
    bid = os.path.join(tag, "build_id.txt")                 # written by tools/pmc.sh: the profiled library
    build = open(bid).read().strip() if os.path.exists(bid) else None
    return {"kernel_regex": pattern, "source": tag, "build_id": build, "kernels": kernels,
            "combined": {"dispatches": dict(cnt), "counters": comb, "derived": derived(comb)}}


def main():
    tag = sys.argv[1]
    pattern = sys.argv[2] if len(sys.argv) > 2 else PRODUCTION_FAMILY
    print(json.dumps(summarise(tag, pattern), indent=1))


if __name__ == "__main__":
    main()
