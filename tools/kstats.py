"""Print a rocprofv3 kernel_stats.csv as one line per kernel (name, calls, avg/min/max us)."""
import csv
import sys

for f in sys.argv[1:]:
    print("==", f)
    for r in csv.DictReader(open(f)):
        n = r["Name"].split("(")[0]
        print(f'{n[:44]:44s} calls={r["Calls"]:>4} avg_us={float(r["AverageNs"])/1e3:9.1f} '
              f'min_us={float(r["MinNs"])/1e3:9.1f} max_us={float(r["MaxNs"])/1e3:9.1f}')
