"""Summarize tools/prof_quick.sh output: per-kernel avg duration + SQ counters per wave."""
import collections
import csv
import glob
import sys

out = sys.argv[1]
st = glob.glob(f"{out}/trace/**/*kernel_stats.csv", recursive=True)
for r in csv.DictReader(open(st[0])):
    print(f"{r['Name'][:60]:60s} calls {r['Calls']:>4s} avg_us {float(r['AverageNs'])/1e3:8.1f} pct {float(r['Percentage']):5.1f}")
acc = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for f in glob.glob(f"{out}/sq*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:40]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[(k, r["Counter_Name"])] += 1
for k, d in acc.items():
    if "apply" not in k and "radix" not in k:
        continue
    waves = d.get("SQ_WAVES", 1)
    print(k, {c: round(v / waves, 1) for c, v in sorted(d.items()) if c != "SQ_WAVES"}, "waves/dispatch",
          waves / cnt[(k, "SQ_WAVES")])
