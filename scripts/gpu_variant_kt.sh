#!/bin/bash
# per-variant kernel traces (rocprofv3 --kernel-trace --stats) of scripts/decode_loop.py
#   bash scripts/gpu_variant_kt.sh TAG CONFIG N [STREAMS]
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
for lib in .tmp/exp/lib_*.so; do
  v=$(basename $lib .so)
  JAAD_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $T/$v -o kt --output-format csv -- python3 scripts/decode_loop.py $2 $3 ${4:-0} > $T/$v.log 2>&1 || exit $?
done
