#!/bin/bash
# Round-end style check on the box: gpu tests (non-slow), smoke(), then the default bench line.
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m "gpu and not slow" > gpurun_out/check_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/check_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/check_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc" >> gpurun_out/check_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/check_bench.log 2>&1
rc=$?; echo "bench rc=$rc" >> gpurun_out/check_bench.log
exit $rc
