#!/bin/bash
# Round 5: PCIe roofs of the box beside the host-entry rates (C2, C4, C5 bench lines, e2e only).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 120 python3 -u scripts/pcie_probe.py > $T/pcie.log 2>&1 || exit 1
for c in 2 4 5; do timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-host --steps 5 --warmup 2 > $T/e2e_bench_c$c.log 2>&1 || exit 1; done
timeout -k 10 120 python3 -u scripts/pcie_probe.py >> $T/pcie.log 2>&1
