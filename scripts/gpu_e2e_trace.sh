#!/bin/bash
# Host-buffer entry: frames/s, then a kernel + memory-copy trace of the same run (overlap of the
# pieces' H2D copies, kernels and D2H copies).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u scripts/e2e_host.py > gpurun_out/e2e_host.log 2>&1 && \
JAAD_E2E_ITERS=2 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/e2e_trace -o e2e -- python3 -u scripts/e2e_host.py > gpurun_out/e2e_trace.log 2>&1
