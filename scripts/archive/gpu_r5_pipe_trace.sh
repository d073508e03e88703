#!/bin/bash
# Round 5: C5 host-entry pipeline timeline -- host per-piece timings and a kernel + copy trace.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
JAAD_E2E_CONFIG=5 JAAD_TRACE_HOST=1 timeout -k 10 300 python3 -u scripts/e2e_host.py > $T/e2e_c5.log 2>&1 &&
JAAD_E2E_CONFIG=5 JAAD_E2E_ITERS=2 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $T/trace -o e2e -- python3 -u scripts/e2e_host.py > $T/e2e_trace.log 2>&1
for c in 4 5; do timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-host --steps 5 --warmup 2 > $T/e2e_bench_c$c.log 2>&1 || exit 1; done
