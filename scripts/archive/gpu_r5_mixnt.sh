#!/bin/bash
# Round 5: ps_mix nontemporal QMF-row loads/stores (JAAD_MIX_NT) against the same build without:
# PS parity with the variant, same-process A/B on C5, kernel traces.   bash scripts/gpu_r5_mixnt.sh TAG
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
JAAD_LIB=$PWD/.tmp/exp2/lib_nt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_ps.py -m gpu -x -q --timeout 200 --timeout-method thread > $T/parity_nt.log 2>&1 || exit $?
timeout -k 10 300 python -u scripts/ab_inproc.py 5 12 10 .tmp/exp2/lib_base.so .tmp/exp2/lib_nt.so > $T/ab.txt 2>&1 || exit $?
for v in base nt; do
  JAAD_LIB=$PWD/.tmp/exp2/lib_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $T/kt5/$v -o kt --output-format csv -- python3 scripts/decode_loop.py 5 20 256 > $T/kt5_$v.log 2>&1 || exit $?
done
