#!/bin/bash
# LC parity tests, bench line, one PMC pass (LDS / VALU counters) on the default workload.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/q; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/q/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/q/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu ${BENCH_ARGS} > gpurun_out/q/bench.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAIT_ANY -d gpurun_out/q/pmc -o pmc --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu ${BENCH_ARGS} > gpurun_out/q/pmc.log 2>&1
rc=$?
python3 - <<'PY' >> gpurun_out/q/pmc.log 2>&1
import csv, glob, collections
acc = collections.defaultdict(list)
for f in glob.glob("gpurun_out/q/pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "lc_decode" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:24s} {sum(v)/len(v):16.0f}")
PY
exit $rc
