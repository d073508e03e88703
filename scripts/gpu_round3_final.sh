#!/bin/bash
# Round-3 closing checks: the whole GPU suite (incl. the full-size batches), smoke(), then the clean C2
# kernel trace + PMC passes (scripts/gpu_prof.sh, bench without the host-buffer leg).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > gpurun_out/final_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/final_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || exit $?
bash scripts/gpu_prof.sh round3_final || exit $?
bash scripts/gpu_e2e_trace.sh
