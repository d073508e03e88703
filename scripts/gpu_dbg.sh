#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python scripts/debug_lc.py ${1:-2} > gpurun_out/dbg.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/dbg.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 420 python -m pytest tests/test_gpu_parity.py -q -m "gpu and not slow" > gpurun_out/pytest.log 2>&1; rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 240 python bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc" >> gpurun_out/bench.log
