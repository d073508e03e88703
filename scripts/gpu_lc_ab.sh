#!/bin/bash
# LC kernel: parity tests, then A/B timing of the library variants in .tmp/exp (same box,
# alternating variants so clock drift hits all alike).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
ROUNDS=${1:-3}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robustness.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lc_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/lc_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u scripts/time_variants.py 2 $ROUNDS > gpurun_out/lc_ab.log 2>&1 && \
timeout -k 10 400 python -u scripts/time_variants.py 3 $ROUNDS >> gpurun_out/lc_ab.log 2>&1
