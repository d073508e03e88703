#!/bin/bash
# round 4: decorrelator roles rebalanced (JAAD_DECOR_REBAL: transient ratio on the transient wave,
# QMF delay lines on the hybrid link-2 wave) -- PS parity of the variant, C5 kernel traces of both,
# per-role stamps of the variant
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/r4rebal; mkdir -p $T; export TMPDIR=/tmp
JAAD_LIB=$PWD/.tmp/exp/lib_b_rebal.so timeout -k 10 600 python -u -m pytest tests/test_gpu_ps.py tests/test_frame_status.py -m gpu -x -q --timeout 300 --timeout-method thread > $T/parity.log 2>&1
rc=$?; echo "parity rc=$rc" >> $T/parity.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_variant_kt.sh r4rebal/kt5 5 30 256 || exit $?
JAAD_LIB=$PWD/.tmp/exp_st/lib_c_rebal_st.so timeout -k 10 200 python3 scripts/decor_stamps.py > $T/stamps.txt 2>&1
