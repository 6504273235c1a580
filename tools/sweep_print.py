"""Print a tools/r02_async.sh sweep: variant, spp per call, Msamples/s, ms per step."""
import json
import sys

v = None
for line in open(sys.argv[1]):
    line = line.strip()
    if not line.startswith("{"):
        continue
    d = json.loads(line)
    if "variant" in d:
        v = (d["variant"], d.get("spp"))
        continue
    print(v, d["value"], d["ms_per_step"])
