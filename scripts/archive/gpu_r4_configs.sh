#!/bin/bash
# round 4: bench lines for C2..C5 (settled), then the rocprof trace + PMC passes of C3, C4, C5
# (profiles/current_c<config>.json is each bench line's traffic source)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4cfg; export TMPDIR=/tmp
for c in 2 3 4 5; do
  timeout -k 10 400 python3 bench.py --config $c > gpurun_out/r4cfg/bench_c$c.json 2> gpurun_out/r4cfg/bench_c$c.err || exit $?
done
for c in 3 4 5; do bash scripts/gpu_prof.sh round4a_c$c $c || exit $?; done
