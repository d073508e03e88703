#!/bin/bash
# round 4: PS parity on the product library (pipelined decorrelator), kernel traces of C5 per
# variant, per-role stamps
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/r4pipe; mkdir -p $T; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ps.py tests/test_frame_status.py tests/test_gpu_sbr.py -m gpu -x -q --timeout 300 --timeout-method thread > $T/ps_parity.log 2>&1
rc=$?; echo "parity rc=$rc" >> $T/ps_parity.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_variant_kt.sh r4pipe_kt 5 30 256 || exit $?
JAAD_LIB=$PWD/.tmp/exp/lib_d_stamps.so timeout -k 10 200 python3 scripts/decor_stamps.py > $T/stamps.txt 2>&1
