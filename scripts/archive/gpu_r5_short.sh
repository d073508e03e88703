#!/bin/bash
# Round 5: C3 short windows in lockstep -- GPU suite, same-process A/B (C3, C2) vs the previous library.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $T/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $T/tests.log; [ $rc -eq 0 ] || exit $rc
for c in 3 2; do
  timeout -k 10 300 python -u scripts/ab_inproc.py $c 6 10 .tmp/exp/lib_prev.so .tmp/exp/lib_short2.so .tmp/exp/lib_short3.so > $T/ab_c$c.log 2>&1 || exit 1
done
