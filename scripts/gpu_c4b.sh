#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_sbr.py -x -q > gpurun_out/sbr_pytest.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c4prof -o c4 --output-format csv -- python3 bench.py --config 4 --steps 5 --warmup 2 --no-cpu > gpurun_out/c4_prof.log 2>&1
rc=$?
find gpurun_out/c4prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/c4_kernel_stats.csv \;
exit $rc
