#!/bin/bash
# Round 5: LC issue-priority variants -- same-process A/B (C2, C3) and per-wave lifetimes.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 240 python -u scripts/ab_inproc.py 2 6 20 .tmp/exp/lib_base.so .tmp/exp/lib_rank.so > $T/ab_c2.log 2>&1 &&
timeout -k 10 240 python -u scripts/ab_inproc.py 3 6 20 .tmp/exp/lib_base.so .tmp/exp/lib_rank.so > $T/ab_c3.log 2>&1 &&
for lib in wtbase wtrank; do
  echo "== $lib" >> $T/wavetime.log
  JAAD_LIB=$PWD/.tmp/exp/lib_$lib.so timeout -k 10 120 python -u scripts/wavetime.py 2 >> $T/wavetime.log 2>&1 || exit 1
done
