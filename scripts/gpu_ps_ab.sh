#!/bin/bash
# C5: A/B timing (PCM hash) and kernel traces of the library variants in .tmp/exp.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/time_variants.py 5 ${1:-3} > gpurun_out/ps_ab.log 2>&1 || exit $?
CFGS=5 bash scripts/gpu_sbr_kt.sh
