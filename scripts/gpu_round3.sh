#!/bin/bash
# Round-3 measurements: bench lines C2..C5 (CPU baseline on C2), kernel-trace stats for C2 / C4 / C5,
# then the C2 PMC passes (scripts/gpu_prof.sh).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > gpurun_out/r3_bench_c2.log 2>&1 || exit $?
for c in 3 4 5; do
  timeout -k 10 400 python3 bench.py --config $c --no-cpu --no-e2e > gpurun_out/r3_bench_c$c.log 2>&1 || exit $?
done
for c in 4 5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3prof_c$c -o c$c --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu --no-e2e > gpurun_out/r3prof_c$c.log 2>&1 || exit $?
done
bash scripts/gpu_prof.sh round3
