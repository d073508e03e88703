#!/bin/bash
# Round 5: SBR/PS host-entry pipeline -- GPU suite, then e2e rates per piece count (C4, C5) and bench lines.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $T/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $T/tests.log; [ $rc -eq 0 ] || exit $rc
for c in 4 5; do
  for np in 4 6 8 12; do
    JAAD_SBR_PIECES=$np timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-host --steps 5 --warmup 2 > $T/e2e_c${c}_p$np.log 2>&1 || exit 1
  done
done
