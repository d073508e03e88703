#!/bin/bash
# LC packed-FP32 IMDCT: parity, then alternating A/B of the scalar and packed builds (C2, C3).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robustness.py tests/test_parse.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lc_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/lc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/time_variants.py 2 3 > gpurun_out/lc_ab.log 2>&1 && \
timeout -k 10 300 python -u scripts/time_variants.py 3 2 >> gpurun_out/lc_ab.log 2>&1
