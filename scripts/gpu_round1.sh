#!/bin/bash
# First GPU bring-up: parity tests, then a short bench (only if the tests did not crash/hang).
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests/test_gpu_parity.py -x -q -m "gpu and not slow" > gpurun_out/r1_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r1_pytest.log
case $rc in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit $rc;; esac
timeout -k 10 240 python bench.py --steps 10 --warmup 3 > gpurun_out/r1_bench.log 2>&1
rc=$?
echo "bench rc=$rc" >> gpurun_out/r1_bench.log
exit $rc
