#!/bin/bash
# A longer randomised parity soak with another seed (tests/test_gpu_soak.py).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
SECS=${1:-600}; SEED=${2:-7}
JAAD_SOAK_SEED=$SEED JAAD_SOAK_SECONDS=$SECS timeout -k 10 $(( SECS + 200 )) python -u -m pytest tests/test_gpu_soak.py -m gpu -x -q -s --timeout $(( SECS + 150 )) --timeout-method thread > gpurun_out/soak_long.log 2>&1
rc=$?; echo "soak rc=$rc" >> gpurun_out/soak_long.log; exit $rc
