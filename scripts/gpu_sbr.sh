#!/bin/bash
# SBR bring-up: SBR parity tests then the LC regression tests.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_sbr.py -x -q > gpurun_out/sbr_pytest.log 2>&1
rc=$?; echo "sbr pytest rc=$rc" >> gpurun_out/sbr_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python -m pytest tests -x -q -m "gpu and not slow" --deselect tests/test_gpu_sbr.py > gpurun_out/lc_pytest.log 2>&1
rc2=$?; echo "lc pytest rc=$rc2" >> gpurun_out/lc_pytest.log
exit $(( rc > rc2 ? rc : rc2 ))
