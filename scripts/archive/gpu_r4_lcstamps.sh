#!/bin/bash
# round 4: LC per-phase stamps (JAAD_STAMPS build) on a settled clock
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
JAAD_LIB=$PWD/.tmp/exp/lib_s_stamps.so timeout -k 10 200 python -u scripts/stamps.py 2 > gpurun_out/stamps_r4.log 2>&1
