"""Summarise the output of the PMC sessions (tools/plans/history_r1_r4.txt == pmc.sh ==): one row per kernel dispatch (lab passes), counters merged."""
import collections
import csv
import glob
import json
import sys

tag = sys.argv[1]
rows = collections.OrderedDict()
for d in sorted(glob.glob(f"gpurun_out/{tag}_pmc*/p_counter_collection.csv")):
    seen = collections.Counter()
    for r in csv.DictReader(open(d)):
        name = r["Kernel_Name"]
        if "onesweep" not in name and "copy" not in name and "hist" not in name:
            continue
        key = (name.split("(")[0][-60:], seen[(name, r["Counter_Name"])])
        seen[(name, r["Counter_Name"])] += 1
        rows.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
out = {f"{k[0]}#{k[1]}": v for k, v in rows.items()}
json.dump(out, open(f"gpurun_out/{tag}_pmc_summary.json", "w"), indent=1)
for k, v in out.items():
    print(k)
    print("   ", ", ".join(f"{a}={b:.4g}" for a, b in sorted(v.items())))
