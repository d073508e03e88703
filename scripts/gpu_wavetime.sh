#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/wavetime.log
for lib in .tmp/wt/lib_*.so; do
  echo "== $lib" >> gpurun_out/wavetime.log
  JAAD_LIB=$PWD/$lib timeout -k 10 120 python -u scripts/wavetime.py 2 >> gpurun_out/wavetime.log 2>&1 || exit 1
done
