#!/bin/bash
# Round 5: launch pipeline (run-aligned for SBR, time slices for PS) -- GPU suite, PCIe roofs, e2e C2/C4/C5 x3.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $T/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $T/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u scripts/pcie_probe.py > $T/pcie.log 2>&1 || exit 1
for k in 1 2 3; do for c in 4 5 2; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-host --steps 3 --warmup 1 > $T/e2e_c${c}_$k.log 2>&1 || exit 1
done; done
