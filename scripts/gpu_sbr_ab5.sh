#!/bin/bash
# SBR: GPU test suite, then 5 alternating rounds of the .tmp/exp library variants on C4 (and 2 on C5).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/time_variants.py 4 5 > gpurun_out/sbr_ab.log 2>&1 && \
timeout -k 10 400 python -u scripts/time_variants.py 5 2 >> gpurun_out/sbr_ab.log 2>&1
