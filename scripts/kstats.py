"""Short per-call table of a rocprofv3 kernel_stats.csv: kernel name, calls,
average and total per step (total / steps).  usage: kstats.py CSV [steps]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
for r in rows:
    n = r["Name"].replace("(anonymous namespace)", "anon")
    m = re.search(r"::(\w+)(<[^(]*>)?\(", n)
    if "rocprim" in n:
        short = "rocprim " + ("histogram" if "histogram" in n else "onesweep" if "onesweep" in n else n[:40])
    else:
        short = (m.group(1) + (m.group(2) or "")) if m else n[:60]
    print(f'{int(r["Calls"]):5d} avg {float(r["AverageNs"]) / 1e3:9.1f} us  per-step {float(r["TotalDurationNs"]) / steps / 1e3:9.1f} us  {short[:70]}')
