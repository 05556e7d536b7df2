"""Per-kernel means of the PMC counters in one rocprofv3 --pmc output dir:
python scripts/pmc_kv.py <dir> <kernel substring> [first_dispatch last_dispatch]"""
import csv
import glob
import sys
from collections import defaultdict

d, sub = sys.argv[1], sys.argv[2]
lo = int(sys.argv[3]) if len(sys.argv) > 3 else 0
hi = int(sys.argv[4]) if len(sys.argv) > 4 else 1 << 60
f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
vals = defaultdict(dict)
for r in csv.DictReader(open(f)):
    if sub not in r["Kernel_Name"]:
        continue
    vals[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
ids = sorted(vals)
sel = [i for k, i in enumerate(ids) if lo <= k <= hi]
keys = sorted({c for i in sel for c in vals[i]})
print(f"{len(sel)} of {len(ids)} dispatches")
for c in keys:
    xs = [vals[i].get(c, 0.0) for i in sel]
    print(f"{c} mean {sum(xs) / len(xs):.4g}  per-dispatch {[round(x) for x in xs[:12]]}")
