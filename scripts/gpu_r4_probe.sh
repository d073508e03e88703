#!/bin/bash
# round 4 probe: instruction-cost micro-benchmark, LC parity + same-call A/B of .tmp/exp, full GPU suite
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4probe; export TMPDIR=/tmp
timeout -k 10 120 .tmp/valu_rate 2048 > gpurun_out/r4probe/valu_rate4.txt 2>&1 || exit $?
bash scripts/gpu_lc_ab.sh 3 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4probe/gpu_suite.log 2>&1
