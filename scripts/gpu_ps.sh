#!/bin/bash
# PS: parity tests (PS, then SBR regression + golden), then the C5 bench line and kernel-trace stats.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_ps.py -q -x > gpurun_out/ps_pytest.log 2>&1
rc=$?; echo "ps pytest rc=$rc" >> gpurun_out/ps_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -m pytest tests/test_gpu_sbr.py tests/test_golden.py -x -q > gpurun_out/sbr_pytest.log 2>&1 || exit $?
timeout -k 10 400 python3 bench.py --config 5 --steps 10 --warmup 3 > gpurun_out/c5_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c5prof -o c5 --output-format csv -- python3 bench.py --config 5 --steps 5 --warmup 2 --no-cpu > gpurun_out/c5_prof.log 2>&1 || exit $?
find gpurun_out/c5prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/c5_kernel_stats.csv \;
