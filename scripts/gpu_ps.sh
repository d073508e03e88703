#!/bin/bash
# PS bring-up: PS parity tests, then the SBR regression tests.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_ps.py -q > gpurun_out/ps_pytest.log 2>&1
rc=$?; echo "ps pytest rc=$rc" >> gpurun_out/ps_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 600 python -m pytest tests/test_gpu_sbr.py -x -q > gpurun_out/sbr_pytest.log 2>&1
rc2=$?; echo "sbr pytest rc=$rc2" >> gpurun_out/sbr_pytest.log
exit $(( rc > rc2 ? rc : rc2 ))
