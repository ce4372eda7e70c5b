"""Print a rocprofv3 kernel_stats.csv as 'mean us x calls name' lines: python tools/kstats.py CSV..."""
import csv
import re
import sys

for path in sys.argv[1:]:
    print("==", path)
    for r in csv.DictReader(open(path)):
        name = re.sub(r"\(.*", "", r["Name"])[:90]
        print(f"{float(r['AverageNs']) / 1e3:10.1f} us x{int(r['Calls']):>5}  {name}")
