"""Per-kernel average times (us) of every variant directory under gpurun_out/TAG/kt<config>/."""
import csv
import sys
from pathlib import Path

root = Path(sys.argv[1])
for kt in sorted(root.glob("kt[0-9]")):
    vs = sorted(d.name for d in kt.iterdir() if d.is_dir())
    rows = {}
    for v in vs:
        for r in csv.DictReader(open(kt / v / "kt_kernel_stats.csv")):
            n = r["Name"].replace("jaad::(anonymous namespace)::", "").replace("void ", "").replace("jaad::", "")[:36]
            rows.setdefault(n, {})[v] = float(r["AverageNs"]) / 1000
    print(kt.name, "  ".join(f"{v:>10s}" for v in vs))
    for n, d in rows.items():
        print(f"  {n:36s}", "  ".join(f"{d.get(v, 0):10.1f}" for v in vs))
