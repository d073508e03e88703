#!/bin/bash
# Round 6: the +-1 LSB instantiation -- its GPU tests, then same-process A/Bs against the exact kernel
# (C2, C3) with the PCM difference of each context to the first.
#   bash scripts/gpu_r6_prec.sh TAG [extra libs for the A/B...]
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; shift; mkdir -p $T; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_precision.py -m gpu -x -q -s --timeout 300 --timeout-method thread > $T/prec_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $T/prec_tests.log; [ $rc -eq 0 ] || exit $rc
L=jaadec_amd/libjaadgpu.so
for c in 2 3; do
  timeout -k 10 300 python -u scripts/ab_inproc.py $c 8 20 $L $L@precision=1 "$@" > $T/ab_c$c.log 2>&1 || exit $?
done
