#!/bin/bash
# SBR + PS parity, then C4/C5 bench lines and kernel-trace stats.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_ps.py tests/test_gpu_sbr.py tests/test_golden.py tests/test_decoder_api.py -m gpu -q -x > gpurun_out/sbrps_pytest.log 2>&1 || exit $?
for c in 4 5; do
  timeout -k 10 400 python3 bench.py --config $c > gpurun_out/bench_c$c.log 2>&1 || exit $?
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c${c}prof -o c$c --output-format csv -- python3 bench.py --config $c --steps 5 --warmup 2 --no-cpu > gpurun_out/c${c}_prof.log 2>&1 || exit $?
  find gpurun_out/c${c}prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/c${c}_kernel_stats.csv \;
done
