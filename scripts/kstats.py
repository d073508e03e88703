"""Per-kernel average durations from a rocprofv3 kernel_stats.csv: python scripts/kstats.py FILE"""
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    print(f"{r['Name'][:70]:70s} {float(r['AverageNs'])/1e3:10.1f} us  x{r['Calls']}")
