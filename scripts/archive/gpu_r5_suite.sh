#!/bin/bash
# Round 5: the whole GPU suite (verbose names, per-test timeout), then smoke().
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -s > $T/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $T/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $T/smoke.log 2>&1
