#!/bin/bash
# SBR/PS parity tests, then C4/C5 kernel-trace stats.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_sbr.py tests/test_gpu_ps.py tests/test_golden.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/sbr_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/sbr_tests.log; [ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/sbr_k.txt
for c in 4 5; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sk$c -o t --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu > gpurun_out/sk$c.log 2>&1 || exit $?
  echo "== C$c $(tail -1 gpurun_out/sk$c.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" >> gpurun_out/sbr_k.txt
  python3 scripts/kstats.py $(find gpurun_out/sk$c -name "*kernel_stats.csv" | head -1) >> gpurun_out/sbr_k.txt
done
