#!/bin/bash
# LC parity tests, then per-kernel PMC passes and kernel stats on C4 / C5 (SBR/PS kernels).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robustness.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/lc_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/lc_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_pmc_c4.sh || exit $?
bash scripts/gpu_sbr_prof.sh
