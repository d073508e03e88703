#!/bin/bash
# Round 5: sbr_synthesis nontemporal input-row loads (JAAD_SYN_NT) against the same build without:
# SBR/PS parity with the variant, same-process A/B on C4 and C5, kernel traces.
#   bash scripts/gpu_r5_synnt.sh TAG
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
JAAD_LIB=$PWD/.tmp/exp2/lib_synnt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_sbr.py tests/test_gpu_ps.py -m gpu -x -q --timeout 200 --timeout-method thread > $T/parity_synnt.log 2>&1 || exit $?
for c in 4 5; do
  timeout -k 10 300 python -u scripts/ab_inproc.py $c 12 10 .tmp/exp2/lib_base.so .tmp/exp2/lib_synnt.so > $T/ab_c$c.txt 2>&1 || exit $?
done
for c in 4 5; do
  s=128; [ $c = 5 ] && s=256
  for v in base synnt; do
    JAAD_LIB=$PWD/.tmp/exp2/lib_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $T/kt$c/$v -o kt --output-format csv -- python3 scripts/decode_loop.py $c 20 $s > $T/kt${c}_$v.log 2>&1 || exit $?
  done
done
