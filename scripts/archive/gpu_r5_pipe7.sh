#!/bin/bash
# Round 5: C4 host-entry pipeline timeline (host per-piece timings, kernel + copy trace).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
JAAD_E2E_CONFIG=4 JAAD_TRACE_HOST=1 JAAD_E2E_ITERS=3 timeout -k 10 300 python3 -u scripts/e2e_host.py > $T/e2e_c4.log 2>&1 &&
JAAD_E2E_CONFIG=4 JAAD_E2E_ITERS=2 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $T/trace -o e2e -- python3 -u scripts/e2e_host.py > $T/e2e_trace.log 2>&1
