"""HBM traffic per launch of the fused bounce kernel (k_bounce0 / k_bounce / k_tail,
production build) from the separate FETCH_SIZE and WRITE_SIZE passes of tools/pmc.sh.

    python tools/pmc_traffic.py gpurun_out/TAG [out.json]   (default profiles/pmc_traffic.json)

Correction per MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) counts half the bytes of a wide
coalesced read on gfx950 -> x2; WRITE_SIZE (KiB) is exact for 16-B-per-lane stores.
bench.py reports the result as roofline.traffic (per launch, like roofline.achieved).
"""
import csv
import glob
import json
import os
import re
import sys

FAMILY = re.compile(r"k_(bounce|tail|march)<\d+, false|k_raygen<false>")   # every bounce-family launch bench.py counts


def per_launch(tag_dir, counter):
    total, dispatches = 0.0, set()
    for f in sorted(glob.glob(os.path.join(tag_dir, "p*", "*counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter or not FAMILY.search(row["Kernel_Name"]):
                continue
            total += float(row["Counter_Value"])
            dispatches.add((f, row["Dispatch_Id"]))
    return (total * 1024.0 / len(dispatches), len(dispatches)) if dispatches else (None, 0)


def main():
    tag = sys.argv[1].rstrip("/")
    out = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                                             "profiles", "pmc_traffic.json")
    fetch, nf = per_launch(tag, "FETCH_SIZE")
    write, nw = per_launch(tag, "WRITE_SIZE")
    if fetch is None or write is None:
        raise SystemExit("no FETCH_SIZE/WRITE_SIZE rows for the bounce kernels")
    res = {"kernel": "bounce family: k_bounce (bounce 0 and later) + k_tail, and k_raygen + k_march for marched "
                     "worlds; production build",
           "hbm_bytes_per_launch": round(2.0 * fetch + write),
           "fetch_bytes_x2_per_launch": round(2.0 * fetch), "write_bytes_per_launch": round(write),
           "dispatches": {"FETCH_SIZE": nf, "WRITE_SIZE": nw},
           "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes (tools/pmc.sh), {os.path.relpath(os.path.abspath(tag), os.path.abspath('gpurun_out'))}; "
                     "FETCH_SIZE x2 (gfx950)"}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
