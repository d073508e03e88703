#!/bin/bash
# per-role busy ticks of the decorrelator block (JAAD_DECOR_STAMPS build)
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/r4stamps; mkdir -p $T; export TMPDIR=/tmp
JAAD_LIB=$PWD/.tmp/exp/lib_d_stamps.so timeout -k 10 200 python3 scripts/decor_stamps.py > $T/stamps.txt 2>&1
