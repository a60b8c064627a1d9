"""Our kernels from a rocprofv3 kernel_stats.csv (torch kernels omitted)."""
import csv
import glob
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    n = r["Name"].replace("(anonymous namespace)::", "")
    if "at::native" in n or "rocclr" in n:
        continue
    print(f"{n[:50]:52s} calls={r['Calls']:>5s} avg_us={float(r['AverageNs']) / 1e3:8.1f}")
