#!/bin/bash
# A/B timing of the library variants in .tmp/exp on C2 (no parity tests: variants may be partial)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/time_variants.py 2 > gpurun_out/lc_ab.log 2>&1 && \
timeout -k 10 300 python -u scripts/time_variants.py 2 >> gpurun_out/lc_ab.log 2>&1
