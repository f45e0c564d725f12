"""Print a rocprofv3 kernel-stats CSV compactly.  Usage: python tools/kstats.py <run_kernel_stats.csv>..."""
import csv
import sys

for f in sys.argv[1:]:
    print(f)
    for r in csv.DictReader(open(f)):
        print(f"  {r['Name'][:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs']) / 1e3:9.1f} us  max {float(r['MaxNs']) / 1e3:9.1f}")
