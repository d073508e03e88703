#!/bin/bash
# Kernel-trace stats of C4 per library variant in .tmp/exp (JAAD_LIB), to split the SBR time per kernel.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/hft; export TMPDIR=/tmp
for lib in .tmp/exp/lib_*.so; do
  n=$(basename $lib .so)
  export JAAD_LIB=$PWD/$lib
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/hft/$n -o t --output-format csv -- python3 bench.py --config 4 --steps 6 --warmup 2 --no-cpu > gpurun_out/hft/$n.log 2>&1 || exit $?
done
