#!/bin/bash
# C5 at the bench's per-GPU size (256 streams x 128 = 32 768 frames): 5 alternating rounds of the
# .tmp/exp library variants.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/time_variants.py 5 5 256 > gpurun_out/c5_ab.log 2>&1
