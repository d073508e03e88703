#!/bin/bash
# round 4 probe: instruction-cost micro-benchmark, then LC parity tests + same-call A/B of .tmp/exp
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4probe; export TMPDIR=/tmp
timeout -k 10 120 .tmp/valu_rate 2048 > gpurun_out/r4probe/valu_rate4.txt 2>&1 || exit $?
bash scripts/gpu_lc_ab.sh 3
