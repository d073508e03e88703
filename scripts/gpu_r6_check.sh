#!/bin/bash
# Round 6: the whole GPU suite on the product library, smoke(), the LC/host-entry GPU tests once more
# on the JAAD_BOUNDS library (exp/lib_bounds.so: every global access of lc_decode_kernel checked,
# a failing check printed), then the C2 bench line.
#   bash scripts/gpu_r6_check.sh TAG
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread > $T/suite.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $T/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $T/smoke.log 2>&1 || exit $?
if [ -f exp/lib_bounds.so ]; then
  JAAD_LIB=$PWD/exp/lib_bounds.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_frame_status.py \
    tests/test_gpu_host_entry.py tests/test_cce.py tests/test_multichannel.py -m gpu -x -q --timeout 300 \
    --timeout-method thread > $T/bounds.log 2>&1
  rc=$?; echo "pytest rc=$rc; JAAD_BOUNDS lines: $(grep -c JAAD_BOUNDS $T/bounds.log)" >> $T/bounds.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 400 python -u bench.py > $T/bench_c2.json 2> $T/bench_c2.err
