#!/bin/bash
# SBR/PS: parity tests, then alternating A/B of the library variants in .tmp/exp (C4, C5).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_sbr.py tests/test_gpu_ps.py tests/test_parse_sbr.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/sbr_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/sbr_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/time_variants.py 4 3 > gpurun_out/sbr_ab.log 2>&1 && \
timeout -k 10 400 python -u scripts/time_variants.py 5 3 >> gpurun_out/sbr_ab.log 2>&1
