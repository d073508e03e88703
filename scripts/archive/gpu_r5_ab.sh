#!/bin/bash
# Round 5: parity of the in-tree build on the SBR/PS/CCE tests, then a same-process A/B of every
# .tmp/exp/lib_*.so on the given configs.   bash scripts/gpu_r5_ab.sh TAG CONFIG...
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; shift; mkdir -p $T; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_sbr.py tests/test_gpu_ps.py tests/test_cce.py tests/test_mc_sbr.py tests/test_sbr_upsample_header.py tests/test_frame_status.py -m gpu -x -q --timeout 200 --timeout-method thread > $T/parity.log 2>&1
rc=$?; echo "parity rc=$rc" >> $T/parity.log; [ $rc -eq 0 ] || exit $rc
for c in "$@"; do
  timeout -k 10 300 python -u scripts/ab_inproc.py $c 8 10 .tmp/exp/lib_*.so > $T/inproc_c$c.log 2>&1 || exit $?
done
