"""Average rocprofv3 counter values per (run dir, kernel) under a directory:
python tools/pmc_summary.py DIR [kernel-substring]"""
import collections
import csv
import glob
import os
import sys

root = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ""
agg = collections.defaultdict(list)
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    run = os.path.relpath(f, root).split(os.sep)[0]
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if sub and sub not in k:
            continue
        agg[(run.split("_", 1)[-1], k[:70], r["Counter_Name"])].append(float(r["Counter_Value"]))
for key in sorted(agg):
    v = agg[key]
    print(f"{key[0]:8s} {key[1]:70s} {key[2]:28s} n={len(v):3d} avg={sum(v) / len(v):16.1f}")
