#!/bin/bash
# Round 5 close: the bench lines of C2..C5 (all legs), then the profiles of the given configs.
#   bash scripts/gpu_r5_final.sh TAG "BENCH_CONFIGS" "PROF_CONFIGS"
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
for c in $2; do
  timeout -k 10 400 python -u bench.py --config $c > $T/bench_c$c.json 2> $T/bench_c$c.err || exit $?
done
for c in $3; do
  bash scripts/gpu_prof.sh $1_c$c $c || exit $?
done
