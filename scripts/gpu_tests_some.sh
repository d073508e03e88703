#!/bin/bash
# A subset of the GPU tests (the files given as arguments), one pytest process.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/some_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/some_tests.log; exit $rc
