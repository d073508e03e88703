#!/bin/bash
# parity of one .tmp/exp variant (or "-"), then a same-process A/B of all .tmp/exp variants
#   bash scripts/gpu_ab_inproc.sh TAG VARIANT BLOCKS PER CONFIG...
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
V=$2; B=$3; P=$4; shift 4
if [ "$V" != "-" ]; then
  JAAD_LIB=$PWD/.tmp/exp/lib_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sbr.py tests/test_frame_status.py -m gpu -x -q --timeout 200 --timeout-method thread > $T/parity_$V.log 2>&1
  rc=$?; echo "parity rc=$rc" >> $T/parity_$V.log
  [ $rc -eq 0 ] || exit $rc
fi
for c in "$@"; do
  timeout -k 10 300 python -u scripts/ab_inproc.py $c $B $P .tmp/exp/lib_*.so > $T/inproc_c$c.log 2>&1 || exit $?
done
