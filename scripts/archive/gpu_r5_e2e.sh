#!/bin/bash
# Round 5: the in-tree build's full GPU suite, then the C4 / C5 bench lines (device + e2e legs).
#   bash scripts/gpu_r5_e2e.sh TAG
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $T/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $T/tests.log; [ $rc -eq 0 ] || exit $rc
for c in 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu --no-host > $T/bench_c$c.json 2> $T/bench_c$c.err || exit $?
done
