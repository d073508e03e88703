#!/bin/bash
# Multichannel / facade GPU tests, then the randomised parity soak (tests/test_gpu_soak.py).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_multichannel.py tests/test_decoder_api.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/mc_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/mc_tests.log; [ $rc -eq 0 ] || exit $rc
JAAD_SOAK_SECONDS=${1:-300} timeout -k 10 $(( ${1:-300} + 200 )) python -u -m pytest tests/test_gpu_soak.py -m gpu -x -q -s --timeout $(( ${1:-300} + 150 )) --timeout-method thread > gpurun_out/soak.log 2>&1
rc=$?; echo "soak rc=$rc" >> gpurun_out/soak.log; exit $rc
