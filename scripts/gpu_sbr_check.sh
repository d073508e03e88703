#!/bin/bash
# SBR / PS GPU parity (incl. coupling and the fallback frames), then the LC stamps + profile.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sbr.py tests/test_gpu_ps.py tests/test_parse_sbr.py -m gpu -x -v --timeout 300 --timeout-method thread -k "not full" > gpurun_out/sbr_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/sbr_tests.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_lc_stamps.sh ${1:-r3a}
