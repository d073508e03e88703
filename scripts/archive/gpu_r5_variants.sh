#!/bin/bash
# Round 5: every .tmp/exp/lib_*.so variant: SBR/PS parity (JAAD_LIB), then kernel traces of
# scripts/decode_loop.py on C4 and C5.   bash scripts/gpu_r5_variants.sh TAG
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
for lib in .tmp/exp/lib_*.so; do
  v=$(basename $lib .so)
  JAAD_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_sbr.py tests/test_gpu_ps.py tests/test_mc_sbr.py -m gpu -x -q --timeout 200 --timeout-method thread > $T/parity_$v.log 2>&1
  rc=$?; echo "parity rc=$rc" >> $T/parity_$v.log; [ $rc -eq 0 ] || exit $rc
done
for c in 4 5; do
  s=128; [ $c = 5 ] && s=256
  for lib in .tmp/exp/lib_*.so; do
    v=$(basename $lib .so)
    JAAD_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $T/kt$c/$v -o kt --output-format csv -- python3 scripts/decode_loop.py $c 20 $s > $T/kt${c}_$v.log 2>&1 || exit $?
  done
done
