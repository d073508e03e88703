#!/bin/bash
# round 4 probe, part 1: instruction-cost micro-benchmark; the GPU suite on the product library;
# same-call A/B of .tmp/exp (scripts/build_variants.py) on C2/C3 (30 launches each, 3 rounds)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4probe; export TMPDIR=/tmp
timeout -k 10 120 .tmp/valu_rate 2048 > gpurun_out/r4probe/valu_rate4.txt 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4probe/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc" >> gpurun_out/r4probe/gpu_suite.log
case $rc in 124|134|137|139) exit $rc;; esac
for c in 2 3; do timeout -k 10 240 python -u scripts/time_variants.py $c 3 > gpurun_out/r4probe/ab_c$c.log 2>&1 || exit $?; done
