#!/bin/bash
# Bench lines for C2 (default), C3, C4, C5 on one GPU.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in 2 3 4 5; do
  timeout -k 10 400 python3 bench.py --config $c > gpurun_out/bench_c$c.log 2>&1 || exit $?
done
