#!/bin/bash
# C5 per-GPU size, 2 alternating rounds of the .tmp/exp variants (timing probes)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/time_variants.py 5 2 256 > gpurun_out/c5_ab.log 2>&1
