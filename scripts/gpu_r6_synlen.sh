#!/bin/bash
# Round 6: SBR synthesis chunk length (JAAD_SYN_FRAMES) vs C4/C5 kernel time (rocprofv3 kernel trace).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
for cfg in 4 5; do
  for n in 3 4 5 6 8; do
    JAAD_SYN_FRAMES=$n timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $T/c${cfg}_n$n -o trace --output-format csv -- python3 bench.py --config $cfg --no-cpu --no-e2e --no-host --steps 20 --warmup 5 > $T/c${cfg}_n$n.log 2>&1 || exit 1
  done
done
