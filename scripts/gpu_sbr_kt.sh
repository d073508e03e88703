#!/bin/bash
# Kernel-trace stats of each library variant in .tmp/exp on the C4 (and C5) workload.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in ${CFGS:-4 5}; do
for lib in .tmp/exp/lib_*.so; do
  n=$(basename $lib .so)
  JAAD_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/kt/c${cfg}_$n -o kt --output-format csv -- python3 scripts/time_variants_child.py $cfg > gpurun_out/kt_c${cfg}_$n.log 2>&1 || exit $?
done
done
