#!/bin/bash
# round 4 close, part 1: the whole -m gpu suite + smoke(), then settled bench lines C2..C5
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/r4close; mkdir -p $T; export TMPDIR=/tmp
bash scripts/gpu_all_tests.sh > $T/suite.log 2>&1
rc=$?; echo "suite rc=$rc" >> $T/suite.log; [ $rc -eq 0 ] || exit $rc
for c in 2 3 4 5; do
  timeout -k 10 400 python3 bench.py --config $c > $T/bench_c$c.json 2> $T/bench_c$c.err || exit $?
done
