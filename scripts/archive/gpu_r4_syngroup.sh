#!/bin/bash
# round 4: synthesis software-pipeline group size (JAAD_SYN_GROUP variants in .tmp/exp) -- parity of
# the largest, then per-variant kernel traces of C4 and C5
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/${TAG:-r4sg}; mkdir -p $T; export TMPDIR=/tmp
JAAD_LIB=$PWD/.tmp/exp/lib_${PARITY_LIB:-g8}.so timeout -k 10 600 python -u -m pytest tests/test_gpu_sbr.py tests/test_gpu_ps.py -m gpu -x -q --timeout 300 --timeout-method thread > $T/parity.log 2>&1
rc=$?; echo "parity rc=$rc" >> $T/parity.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_variant_kt.sh ${TAG:-r4sg}/kt4 4 30 || exit $?
bash scripts/gpu_variant_kt.sh ${TAG:-r4sg}/kt5 5 30 256
