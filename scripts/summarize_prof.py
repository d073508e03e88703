"""Summarize a scripts/gpu_prof.sh output directory into profiles/<tag>.json + .md.

HBM traffic per launch follows MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE
come from separate --pmc passes (units of KiB); on gfx950 FETCH_SIZE reports half of the bytes
of wide (16 B/lane) coalesced streaming reads, so it is doubled; WRITE_SIZE is exact for
16-B-per-lane stores.  The kernel's input stream is dominated by 16-B q loads (~88 % of read
bytes), so the doubling is applied to all of FETCH_SIZE (stated in the summary).
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

KERNEL = "lc_decode_kernel"


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main(prof_dir: str, tag: str, out_dir: str = "profiles"):
    d = Path(prof_dir)
    out = Path(out_dir)
    out.mkdir(exist_ok=True)
    summary = {"tag": tag, "kernel": KERNEL}
    stats = [r for r in rows(d / "trace_kernel_stats.csv") if KERNEL in r["Name"]]
    if stats:
        s = stats[0]
        summary["trace"] = {"name": s["Name"], "calls": int(s["Calls"]), "avg_ns": float(s["AverageNs"]),
                            "min_ns": float(s["MinNs"]), "max_ns": float(s["MaxNs"])}
    pmc = defaultdict(list)
    for f in sorted(d.glob("pmc*_counter_collection.csv")):
        for r in rows(f):
            if KERNEL in r["Kernel_Name"]:
                pmc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in pmc.items()}
    summary["pmc_avg_per_launch"] = avg
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        fetch = avg["FETCH_SIZE"] * 1024 * 2
        write = avg["WRITE_SIZE"] * 1024
        summary["hbm_traffic_bytes_per_launch"] = fetch + write
        summary["hbm_traffic_note"] = "2 x FETCH_SIZE (gfx950 half-count correction) + WRITE_SIZE, KiB -> bytes"
        summary["fetch_bytes"] = fetch
        summary["write_bytes"] = write
    (out / f"{tag}.json").write_text(json.dumps(summary, indent=1))
    # copy the raw stats table too (the committed rocprof summary)
    if (d / "trace_kernel_stats.csv").exists():
        (out / f"{tag}_kernel_stats.csv").write_text((d / "trace_kernel_stats.csv").read_text())
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
