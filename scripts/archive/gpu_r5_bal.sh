#!/bin/bash
# Round 5: LC tail balance -- chunk skew by SIMD slot (JAAD_LC_SKEW) and rank priority (JAAD_PRIO_RANK):
# same-process A/B on C2 / C3, then per-wave lifetimes.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
L=.tmp/exp
for c in 2 3; do
timeout -k 10 300 python -u scripts/ab_inproc.py $c 6 10 $L/lib_cur.so $L/lib_cur.so@JAAD_LC_SKEW=0.03 $L/lib_cur.so@JAAD_LC_SKEW=0.06 $L/lib_cur.so@JAAD_LC_SKEW=0.10 $L/lib_rank.so $L/lib_rank.so@JAAD_LC_SKEW=0.05 > $T/ab_c$c.log 2>&1 || exit 1
done
for v in wt wtrank; do
  echo "== $v" >> $T/wavetime.log
  JAAD_LIB=$PWD/$L/lib_$v.so timeout -k 10 120 python -u scripts/wavetime.py 2 >> $T/wavetime.log 2>&1 || exit 1
done
echo "== wt skew 0.06" >> $T/wavetime.log
JAAD_LC_SKEW=0.06 JAAD_LIB=$PWD/$L/lib_wt.so timeout -k 10 120 python -u scripts/wavetime.py 2 >> $T/wavetime.log 2>&1
