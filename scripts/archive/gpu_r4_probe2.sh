#!/bin/bash
# round 4 probe, part 2: parity of the VOP3-rewritten variants; same-call A/B on C4/C5
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4probe; export TMPDIR=/tmp
for v in c_vop3 d_vop3c; do
  JAAD_LIB=$PWD/.tmp/exp/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sbr.py tests/test_gpu_ps.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r4probe/parity_$v.log 2>&1 || exit $?
done
for c in 4 5; do timeout -k 10 300 python -u scripts/time_variants.py $c 3 > gpurun_out/r4probe/ab_c$c.log 2>&1 || exit $?; done
