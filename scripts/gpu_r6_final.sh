#!/bin/bash
# Round 6 close, part 1: the whole GPU suite, smoke(), the precision tests with their printed
# off-by-one fractions, one randomised parity soak (<= 300 s).   bash scripts/gpu_r6_final.sh TAG
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $T/suite.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $T/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $T/smoke.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest tests/test_gpu_precision.py -m gpu -q -s --timeout 200 --timeout-method thread > $T/precision.log 2>&1 || exit $?
JAAD_SOAK_SECONDS=240 timeout -k 10 330 python -u -m pytest tests/test_gpu_soak.py -m gpu -q -s --timeout 320 --timeout-method thread > $T/soak.log 2>&1
