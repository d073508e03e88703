#!/bin/bash
# Host-buffer entry + SBR chain walker: parity, then the C2 bench line (e2e legs included).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_entry.py tests/test_gpu_sbr.py tests/test_decoder_api.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/host_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/host_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --no-cpu > gpurun_out/host_bench.log 2>&1
