#!/bin/bash
# kernel durations and inter-kernel gaps (rocprofv3 kernel trace) of each .tmp/exp variant on C2
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/lctrace; export TMPDIR=/tmp
for lib in .tmp/exp/lib_*.so; do
  v=$(basename $lib .so); export JAAD_LIB=$PWD/$lib
  timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/lctrace/$v -o tr --output-format csv -- python3 scripts/time_variants_child.py 2 > gpurun_out/lctrace/$v.log 2>&1 || exit 1
done
