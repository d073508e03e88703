#!/bin/bash
# Round 5, stereo pair kernel: same-process A/B against lc_decode_kernel (copies of one build, the
# second with JAAD_LC_PAIR=0; PCM hashes must agree), then the whole GPU suite.
#   bash scripts/gpu_r5_pair.sh TAG [BLOCKS PER]
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
B=${2:-6}; P=${3:-20}
timeout -k 10 240 python -u scripts/ab_inproc.py 2 $B $P .tmp/exp/lib_a.so .tmp/exp/lib_b.so@JAAD_LC_PAIR=0 > $T/ab_c2.log 2>&1 &&
timeout -k 10 240 python -u scripts/ab_inproc.py 3 $B $P .tmp/exp/lib_a.so .tmp/exp/lib_b.so@JAAD_LC_PAIR=0 > $T/ab_c3.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $T/tests.log 2>&1
rc=$?; echo "rc=$rc" >> $T/tests.log; exit $rc
