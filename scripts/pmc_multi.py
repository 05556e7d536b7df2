"""HBM bytes per call of a multi-launch entry point from rocprofv3 --pmc
FETCH_SIZE / WRITE_SIZE passes: the counters of every dispatch whose kernel
name contains one of the given substrings, summed, divided by the number of
dispatches of the anchor kernel (one per call).  gfx950 correction as in
pmc_summary.py: FETCH_SIZE doubled, both in KiB.

usage: pmc_multi.py FETCH_DIR WRITE_DIR k1,k2,.. ANCHOR WORKLOAD_KEY OUT..."""
import csv
import glob
import json
import os
import sys

fetch_dir, write_dir, names, anchor, key = sys.argv[1:6]
outs = sys.argv[6:]
names = names.split(",")


SKIP = int(os.environ.get("SKIP_ANCHORS", "0"))  # set-up calls before the measured ones


def per_call(d, counter):
    vals, calls = {}, set()
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            kn = r["Kernel_Name"]
            did = int(r["Dispatch_Id"])
            if anchor in kn:
                calls.add(did)
            if any(n in kn for n in names):
                vals[did] = vals.get(did, 0.0) + float(r["Counter_Value"])
    # SKIP_ANCHORS = k: the first k anchor dispatches and everything before
    # the k-th are set-up (e.g. the compaction bench's input build and decode)
    if SKIP:
        first = sorted(calls)[SKIP]
        calls = {c for c in calls if c >= first}
        vals = {k: v for k, v in vals.items() if k >= first}
    return sum(vals.values()) / max(1, len(calls)), len(calls)


fk, nf = per_call(fetch_dir, "FETCH_SIZE")
wk, nw = per_call(write_dir, "WRITE_SIZE")
res = {"workload_key": key, "kernels": names, "anchor": anchor, "calls": [nf, nw],
       "fetch_bytes_per_launch": 2 * 1024 * fk, "write_bytes_per_launch": 1024 * wk,
       "hbm_bytes_per_launch": 2 * 1024 * fk + 1024 * wk,
       "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB x 1024; summed over the "
                     "call's launches"}
for o in outs:
    json.dump(res, open(o, "w"), indent=1)
print(json.dumps(res))
