#!/bin/bash
# Closing check: the whole GPU suite + smoke(), the randomised soak, bench lines C2-C5.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_all_tests.sh || exit $?
JAAD_SOAK_SECONDS=${1:-150} timeout -k 10 $(( ${1:-150} + 200 )) python -u -m pytest tests/test_gpu_soak.py -m gpu -x -q -s --timeout $(( ${1:-150} + 150 )) --timeout-method thread > gpurun_out/soak.log 2>&1
rc=$?; echo "soak rc=$rc" >> gpurun_out/soak.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_bench_all.sh
