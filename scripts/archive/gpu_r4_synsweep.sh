#!/bin/bash
# round 4: synthesis chunk-length sweep (JAAD_SYN_FRAMES), kernel traces of C4 and C5
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/r4synsweep; mkdir -p $T; export TMPDIR=/tmp
for c in 4 5; do
  s=0; [ $c = 5 ] && s=256
  for L in 2 3 4 5 6 8; do
    JAAD_SYN_FRAMES=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $T/L${L}_c$c -o kt --output-format csv -- python3 scripts/decode_loop.py $c 30 $s > $T/L${L}_c$c.log 2>&1 || exit $?
  done
done
