#!/bin/bash
# Round 6: bench lines (C2 +-1 LSB = the headline, C2 exact, C3, C4, C5), then the rocprofv3 kernel
# trace + PMC passes of the C2 and C3 bench commands (scripts/gpu_prof.sh).
#   bash scripts/gpu_r6_close.sh TAG
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > $T/bench_c2.json 2> $T/bench_c2.err || exit $?
timeout -k 10 400 python -u bench.py --precision exact --no-e2e --no-host > $T/bench_c2_exact.json 2> $T/bench_c2_exact.err || exit $?
for c in 3 4 5; do
  timeout -k 10 400 python -u bench.py --config $c > $T/bench_c$c.json 2> $T/bench_c$c.err || exit $?
done
bash scripts/gpu_prof.sh $1_c2 2 || exit $?
bash scripts/gpu_prof.sh $1_c3 3
