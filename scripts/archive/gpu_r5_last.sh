#!/bin/bash
# Round 5, last tree: the whole GPU suite and smoke(), then the C5 bench line and its profile.
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
bash scripts/gpu_r5_suite.sh $1 || exit $?
timeout -k 10 400 python -u bench.py --config 5 > $T/bench_c5.json 2> $T/bench_c5.err || exit $?
bash scripts/gpu_prof.sh $1_c5 5
