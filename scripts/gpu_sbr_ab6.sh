#!/bin/bash
# SBR/PS parity tests, then A/B: C4 (3 rounds), C5 at the per-GPU size (3 rounds)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ps.py tests/test_gpu_sbr.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/time_variants.py 4 3 > gpurun_out/sbr_ab.log 2>&1 && \
timeout -k 10 400 python -u scripts/time_variants.py 5 3 256 >> gpurun_out/sbr_ab.log 2>&1
