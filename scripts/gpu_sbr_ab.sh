#!/bin/bash
# SBR/PS: GPU tests, then A/B timing of the library variants in .tmp/exp on C4 and C5.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=${1:-3}
timeout -k 10 600 python -u -m pytest tests/test_gpu_sbr.py tests/test_gpu_ps.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sbr_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/sbr_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/time_variants.py 4 $ROUNDS > gpurun_out/sbr_ab.log 2>&1 && \
timeout -k 10 400 python -u scripts/time_variants.py 5 $ROUNDS >> gpurun_out/sbr_ab.log 2>&1
