"""Print a rocprofv3 kernel_stats.csv as a short table (kernels above 0.3 %)."""
import csv
import sys

for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].replace("(anonymous namespace)::", "")[:44]
    if float(r["Percentage"]) > 0.3:
        print(f"{n:46s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs']) / 1e3:9.1f} "
              f"pct={float(r['Percentage']):5.2f}")
