#!/bin/bash
# round 4 probe: instruction-cost micro-benchmark; the GPU suite on the product library; parity of
# the VOP3-rewritten variants; same-call A/B of .tmp/exp on C2..C5
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4probe; export TMPDIR=/tmp
timeout -k 10 120 .tmp/valu_rate 2048 > gpurun_out/r4probe/valu_rate4.txt 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4probe/gpu_suite.log 2>&1
echo "suite rc=$?" >> gpurun_out/r4probe/gpu_suite.log
for v in c_vop3 d_vop3c; do
  JAAD_LIB=$PWD/.tmp/exp/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sbr.py tests/test_gpu_ps.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r4probe/parity_$v.log 2>&1 || exit $?
done
for c in 2 3 4 5; do timeout -k 10 400 python -u scripts/time_variants.py $c 3 > gpurun_out/r4probe/ab_c$c.log 2>&1 || exit $?; done
