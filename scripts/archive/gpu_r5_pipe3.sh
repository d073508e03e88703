#!/bin/bash
# Round 5: time-sliced launch pipeline -- GPU suite, PCIe roofs, e2e rates (bench C2/C4/C5), C5 host timings.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $T/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $T/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u scripts/pcie_probe.py > $T/pcie.log 2>&1 || exit 1
for c in 4 5 2; do timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-host --steps 5 --warmup 2 > $T/e2e_bench_c$c.log 2>&1 || exit 1; done
JAAD_E2E_CONFIG=5 JAAD_TRACE_HOST=1 JAAD_E2E_ITERS=3 timeout -k 10 300 python3 -u scripts/e2e_host.py > $T/e2e_c5.log 2>&1
