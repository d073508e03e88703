#!/bin/bash
# round 4: SBR slot-state copy with batched float4 loads -- SBR/PS/multichannel parity of the
# product library, then per-variant kernel traces of C4 and C5 (.tmp/exp/lib_*.so)
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/r4state; mkdir -p $T; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sbr.py tests/test_gpu_ps.py tests/test_multichannel.py tests/test_cce.py tests/test_frame_status.py -m gpu -x -q --timeout 300 --timeout-method thread > $T/parity.log 2>&1
rc=$?; echo "parity rc=$rc" >> $T/parity.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_variant_kt.sh r4state/kt4 4 30 || exit $?
bash scripts/gpu_variant_kt.sh r4state/kt5 5 30 256
