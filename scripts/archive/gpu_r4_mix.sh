#!/bin/bash
# round 4: ps_mix_kernel in 8-slot chunks -- PS parity of the product library, then per-variant
# kernel traces of C5 (.tmp/exp/lib_*.so)
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/r4mix; mkdir -p $T; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ps.py tests/test_gpu_sbr.py tests/test_frame_status.py -m gpu -x -q --timeout 300 --timeout-method thread > $T/parity.log 2>&1
rc=$?; echo "parity rc=$rc" >> $T/parity.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_variant_kt.sh r4mix/kt5 5 30 256
