"""Timeline of a rocprofv3 --kernel-trace CSV: per dispatch, kernel time and
the idle gap before it (µs), plus the sum over a selected dispatch range.
python scripts/ktrace_gaps.py <run_kernel_trace.csv> [first last]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
lo = int(sys.argv[2]) if len(sys.argv) > 2 else 0
hi = int(sys.argv[3]) if len(sys.argv) > 3 else len(rows) - 1
prev = None
busy = gaps = 0.0
for i, r in enumerate(rows):
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1000 if prev is not None else 0.0
    if lo <= i <= hi:
        busy += (e - s) / 1000
        gaps += gap if i > lo else 0.0
    print(f"{i:4d} {r['Kernel_Name'][:60]:60s} {(e - s) / 1000:9.2f} us  gap {gap:10.2f} us")
    prev = e
n = hi - lo + 1
print(f"dispatches {lo}..{hi}: {n} kernels, kernel sum {busy:.1f} us ({busy / n:.2f} per kernel), "
      f"gaps between them {gaps:.1f} us, first start to last end {busy + gaps:.1f} us")
