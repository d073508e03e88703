#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python3 scripts/time_variants.py ${1:-2} > gpurun_out/variants.log 2>&1
