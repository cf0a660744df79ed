import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:58]:58s} calls={r['Calls']:>4s} avg_us={float(r['AverageNs'])/1e3:8.1f} min_us={float(r['MinNs'])/1e3:8.1f}")
