#!/bin/bash
# PS parity tests, then C5 A/B at the per-GPU size (256 streams) and at the full job (2048 streams)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ps.py tests/test_gpu_sbr.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/time_variants.py 5 4 256 > gpurun_out/c5_ab.log 2>&1 && \
timeout -k 10 400 python -u scripts/time_variants.py 5 2 >> gpurun_out/c5_ab.log 2>&1
