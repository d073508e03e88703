#!/bin/bash
# Round 5: bench lines of C4 and C5 (device + e2e legs), then kernel stats of the C4 / C5 bench
# runs under rocprofv3.   bash scripts/gpu_r5_state.sh TAG
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
for c in 4 5; do
  timeout -k 10 300 python -u bench.py --config $c --no-cpu --no-host > $T/bench_c$c.json 2> $T/bench_c$c.err || exit $?
done
for c in 4 5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/kt_c$c -o kt --output-format csv -- python3 bench.py --config $c --no-cpu --no-host --no-e2e > $T/kt_c$c.log 2>&1 || exit $?
done
