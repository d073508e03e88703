#!/bin/bash
# round 4: PS mixing inside the decorrelator block -- parity of the product library (PS, SBR,
# frame status), per-variant kernel traces of C5 (.tmp/exp/lib_*.so), per-role stamps
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/r4fuse; mkdir -p $T; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ps.py tests/test_gpu_sbr.py tests/test_frame_status.py -m gpu -x -q --timeout 300 --timeout-method thread > $T/parity.log 2>&1
rc=$?; echo "parity rc=$rc" >> $T/parity.log; [ $rc -eq 0 ] || exit $rc
mkdir -p .tmp/exp_kt && mv .tmp/exp/lib_d_stamps.so .tmp/exp_kt/
bash scripts/gpu_variant_kt.sh r4fuse/kt5 5 30 256 || exit $?
JAAD_LIB=$PWD/.tmp/exp_kt/lib_d_stamps.so timeout -k 10 200 python3 scripts/decor_stamps.py > $T/stamps.txt 2>&1
