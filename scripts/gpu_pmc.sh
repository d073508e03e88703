#!/bin/bash
# One rocprofv3 PMC pass over a short bench run: gpu_pmc.sh TAG "COUNTERS..." [bench args]
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
TAG=$1; CNT=$2; shift 2
timeout -s KILL 90 rocprofv3 --pmc $CNT -d gpurun_out/pmc/$TAG -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu "$@" > gpurun_out/pmc/$TAG.log 2>&1
rc=$?
python3 - "$TAG" <<'PY' >> gpurun_out/pmc/$TAG.log 2>&1
import csv, glob, collections, sys
acc = collections.defaultdict(list)
for f in glob.glob(f"gpurun_out/pmc/{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{k:60s} {c:24s} {sum(v)/len(v):16.0f}")
PY
exit $rc
