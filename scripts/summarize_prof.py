"""Summarize a scripts/gpu_prof.sh output directory into profiles/<tag>.json (+ the kernel stats csv).

    python3 scripts/summarize_prof.py <prof_dir> <tag> [out_dir] [config]

HBM traffic follows MI355X_MICROARCH.md (HBM / rocprofv3): FETCH_SIZE and WRITE_SIZE come from
separate --pmc passes (units of KiB); on gfx950 FETCH_SIZE reports half of the bytes of wide
(16 B/lane) coalesced streaming reads, so it is doubled; WRITE_SIZE is exact for 16-B-per-lane
stores.  C2/C3: the lc_decode_kernel dispatches (its input stream is ~88 % 16-B q loads).  C4/C5
(several kernels per step): the sum over every kernel dispatch of the run divided by the number
of steps (one lc_decode_kernel dispatch per step); their reads are not all 16-B wide, so the
doubling overstates narrower reads (stated in the note).
"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

KERNEL = "lc_decode_kernel"
FRAMES = {2: 65536, 3: 65536, 4: 32768, 5: 32768}


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main(prof_dir: str, tag: str, out_dir: str = "profiles", config: str = "2"):
    cfg = int(config)
    d = Path(prof_dir)
    out = Path(out_dir)
    out.mkdir(exist_ok=True)
    summary = {"tag": tag, "kernel": KERNEL if cfg in (2, 3) else "all kernels of a step", "config": cfg,
               "frames_per_step": FRAMES[cfg]}
    stats = rows(d / "trace_kernel_stats.csv") if (d / "trace_kernel_stats.csv").exists() else []
    lc = [r for r in stats if KERNEL in r["Name"]]
    if lc:
        s = lc[0]
        summary["trace"] = {"name": s["Name"], "calls": int(s["Calls"]), "avg_ns": float(s["AverageNs"]),
                            "min_ns": float(s["MinNs"]), "max_ns": float(s["MaxNs"])}
    if cfg not in (2, 3) and stats:
        summary["trace_all"] = {r["Name"][:80]: {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])} for r in stats}
    per_kernel = defaultdict(list)   # counter -> values of the LC dispatches
    totals = defaultdict(float)      # counter -> sum over every dispatch
    steps = defaultdict(int)         # counter -> LC dispatches seen in that pass
    for f in sorted(d.glob("pmc*_counter_collection.csv")):
        for r in rows(f):
            c = r["Counter_Name"]
            v = float(r["Counter_Value"])
            totals[c] += v
            if KERNEL in r["Kernel_Name"]:
                per_kernel[c].append(v)
                steps[c] += 1
    if cfg in (2, 3):
        avg = {k: sum(v) / len(v) for k, v in per_kernel.items()}
    else:
        avg = {k: totals[k] / steps[k] for k in totals if steps.get(k)}
    summary["pmc_avg_per_launch" if cfg in (2, 3) else "pmc_per_step"] = avg
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        fetch = avg["FETCH_SIZE"] * 1024 * 2
        write = avg["WRITE_SIZE"] * 1024
        summary["hbm_traffic_bytes_per_launch"] = fetch + write
        summary["hbm_traffic_note"] = ("2 x FETCH_SIZE (gfx950 half-count correction) + WRITE_SIZE, KiB -> bytes" +
                                       ("" if cfg in (2, 3) else ", summed over the step's kernels"))
        summary["fetch_bytes"] = fetch
        summary["write_bytes"] = write
    (out / f"{tag}.json").write_text(json.dumps(summary, indent=1))
    if (d / "trace_kernel_stats.csv").exists():
        (out / f"{tag}_kernel_stats.csv").write_text((d / "trace_kernel_stats.csv").read_text())
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
