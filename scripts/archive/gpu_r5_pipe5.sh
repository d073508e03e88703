#!/bin/bash
# Round 5: launch pipeline with gathered q (1D H2D) + strided PCM D2H -- e2e C4/C5 (P 8, 12) + C5 trace.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
for np in 8 12; do for c in 4 5; do
  JAAD_SBR_PIECES=$np timeout -k 10 300 python3 bench.py --config $c --no-cpu --no-host --steps 3 --warmup 1 > $T/e2e_c${c}_p$np.log 2>&1 || exit 1
done; done
JAAD_E2E_CONFIG=5 JAAD_E2E_ITERS=2 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $T/trace -o e2e -- python3 -u scripts/e2e_host.py > $T/e2e_trace.log 2>&1
