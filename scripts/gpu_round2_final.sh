#!/bin/bash
# Round-2 closing measurements: GPU parity suite (incl. the full C2/C4/C5 batches), bench lines
# C2..C5, kernel-trace stats of C4 and C5.  (LC trace + PMC passes: scripts/gpu_prof.sh.)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
for c in 2 3 4 5; do
  timeout -k 10 400 python3 bench.py --config $c > gpurun_out/bench_c$c.log 2>&1 || exit $?
done
for c in 4 5; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c${c}prof -o c$c --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu > gpurun_out/c${c}_prof.log 2>&1 || exit $?
  find gpurun_out/c${c}prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/c${c}_kernel_stats.csv \;
done
