#!/bin/bash
# The whole GPU suite and smoke() (what the driver runs at round end).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/all_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/all_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/all_smoke.log 2>&1
