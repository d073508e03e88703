#!/bin/bash
# C4 and C5 bench lines (no CPU leg) + kernel-trace stats.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in 4 5; do
  timeout -k 10 300 python3 bench.py --config $c --no-cpu > gpurun_out/c${c}_bench.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c${c}prof -o c$c --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu > gpurun_out/c${c}_prof.log 2>&1 || exit $?
  find gpurun_out/c${c}prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/c${c}_kernel_stats.csv \;
done
