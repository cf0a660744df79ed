"""Sum rocprofv3 --pmc counters per kernel (average per dispatch):  python tools/pmc_sum.py <dir> [name-filter]"""
import csv
import glob
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(float))
disp = defaultdict(set)
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if len(sys.argv) > 2 and sys.argv[2] not in k:
            continue
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
for k, c in sorted(acc.items()):
    n = len(disp[k])
    print(k, f"dispatches {n}", " ".join(f"{m}={v / n:.4g}" for m, v in sorted(c.items())))
