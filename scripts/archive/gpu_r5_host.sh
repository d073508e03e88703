#!/bin/bash
# Round 5: GPU suite, then bench lines C2..C5 with the host front-end leg (tools/bench_parse).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $T/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $T/tests.log; [ $rc -eq 0 ] || exit $rc
for c in 2 4 5 3; do
  timeout -k 10 400 python3 bench.py --config $c > $T/bench_c$c.log 2>&1 || exit 1
done
