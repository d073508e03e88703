#!/bin/bash
# LC kernel: parity tests (LC + golden), then the default bench line and a kernel-trace profile.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_decoder_api.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/lc_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/lc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --no-cpu > gpurun_out/lc_bench.log 2>&1
