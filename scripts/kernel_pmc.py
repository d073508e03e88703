"""Per-kernel PMC table from rocprofv3 --pmc pass directories (scripts/gpu_pmc_c4.sh): average of
each counter over the dispatches of each kernel, plus derived ratios (VALU issue share of the
wave cycles, waits, HBM bytes with the gfx950 FETCH_SIZE half-count correction)."""
import csv
import sys
from collections import defaultdict
from pathlib import Path


def main(root: str):
    acc = defaultdict(lambda: defaultdict(list))
    for f in sorted(Path(root).rglob("*counter_collection.csv")):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("jaad::", "")
                acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in sorted(acc.items()):
        a = {n: sum(v) / len(v) for n, v in c.items()}
        wc = a.get("SQ_WAVE_CYCLES", 0) or 1
        line = [f"{k[:44]:44s}", f"waves {a.get('SQ_WAVES', 0):9.0f}"]
        if "SQ_INSTS_VALU" in a and "SQ_WAVES" in a:
            line.append(f"valu/wave {a['SQ_INSTS_VALU'] / a['SQ_WAVES']:8.0f}")
        for n in ("SQ_ACTIVE_INST_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_LDS"):
            if n in a:
                line.append(f"{n[3:]} {a[n] / wc:5.2f}")
        if "FETCH_SIZE" in a:
            line.append(f"fetch {a['FETCH_SIZE'] * 2048 / 1e6:8.1f} MB")
        if "WRITE_SIZE" in a:
            line.append(f"write {a['WRITE_SIZE'] * 1024 / 1e6:8.1f} MB")
        print("  ".join(line))


if __name__ == "__main__":
    main(sys.argv[1])
