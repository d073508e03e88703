#!/bin/bash
# Host-buffer entry: its GPU tests (and bench.run's two-rank path on the HIP engine), then the C2
# end-to-end rates with pageable, registered and jaad_host_alloc buffers (scripts/e2e_host.py).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_host_entry.py tests/test_bench_multirank.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/e2e_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/e2e_tests.log; [ $rc -eq 0 ] || exit $rc
JAAD_E2E_ITERS=9 timeout -k 10 300 python -u scripts/e2e_host.py > gpurun_out/e2e_host.log 2>&1
