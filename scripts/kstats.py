"""Print the top kernels of a rocprofv3 kernel_stats.csv."""
import csv
import sys

for x in list(csv.DictReader(open(sys.argv[1])))[:int(sys.argv[2]) if len(sys.argv) > 2 else 12]:
    print(f"{x['Name'][:64]:64s} calls={x['Calls']:>5s} avg_us={float(x['AverageNs'])/1e3:9.1f} pct={float(x['Percentage']):6.2f}")
