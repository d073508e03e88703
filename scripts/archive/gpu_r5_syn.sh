#!/bin/bash
# Round 5: paired-slot synthesis.  SBR/PS parity with the new build, then a same-process A/B
# (.tmp/exp/lib_base.so vs lib_pair.so) on C4 and C5, then kernel stats of C5.
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_sbr.py tests/test_gpu_ps.py tests/test_cce.py tests/test_mc_sbr.py tests/test_sbr_upsample_header.py -m gpu -x -q --timeout 200 --timeout-method thread > $T/parity.log 2>&1
rc=$?; echo "parity rc=$rc" >> $T/parity.log; [ $rc -eq 0 ] || exit $rc
for c in 4 5; do
  timeout -k 10 300 python -u scripts/ab_inproc.py $c 8 10 .tmp/exp/lib_base.so .tmp/exp/lib_pair.so > $T/inproc_c$c.log 2>&1 || exit $?
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $T/c5 -o kt --output-format csv -- python3 scripts/decode_loop.py 5 30 > $T/c5.log 2>&1
