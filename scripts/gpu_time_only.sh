#!/bin/bash
# Timing of the library variants in .tmp/exp only (ablation builds are not bit-exact): config $1, rounds $2.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/time_variants.py ${1:-4} ${2:-2} > gpurun_out/time_only.log 2>&1
