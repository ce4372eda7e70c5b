"""Mean of every PMC counter per kernel over rocprofv3 --pmc output directories.

python tools/pmc_kernels.py DIR [DIR ...]   (each DIR holds p_counter_collection.csv, possibly
in a subdirectory); prints one block per kernel: dispatches and the mean value per dispatch.
"""
import collections
import csv
import glob
import os
import sys

sums = collections.defaultdict(lambda: collections.defaultdict(float))
counts = collections.defaultdict(lambda: collections.defaultdict(set))
for d in sys.argv[1:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0]
            c = r["Counter_Name"]
            sums[name][c] += float(r["Counter_Value"])
            counts[name][c].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
for name in sorted(sums):
    print(name[-110:])
    for c in sorted(sums[name]):
        n = max(1, len(counts[name][c]))
        print(f"    {c:28s} dispatches={n:4d}  mean={sums[name][c] / n:.6g}")
