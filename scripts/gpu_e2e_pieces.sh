#!/bin/bash
# Host-buffer entry: e2e rate per piece-count variant (.tmp/exp/lib_p*.so, scripts/build_variants.py),
# alternating variants over rounds.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/e2e_pieces.log
for r in 1 2 3; do
  for lib in .tmp/exp/lib_p*.so; do
    echo "== $lib" >> gpurun_out/e2e_pieces.log
    JAAD_LIB=$lib JAAD_E2E_ITERS=7 timeout -k 10 120 python -u scripts/e2e_host.py >> gpurun_out/e2e_pieces.log 2>&1 || exit $?
  done
done
