#!/bin/bash
# Round 6: SBR/PS GPU tests with the fused analysis, then kernel traces of C4/C5 fused vs
# JAAD_SBR_FUSED=0.   bash scripts/gpu_r6_fuse_ab.sh TAG
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_gpu_sbr.py tests/test_gpu_ps.py tests/test_mc_sbr.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $T/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $T/tests.log; [ $rc -eq 0 ] || exit $rc
for cfg in 4 5; do
  for fz in 1 0; do
    JAAD_SBR_FUSED=$fz timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $T/c${cfg}_f$fz -o trace --output-format csv -- python3 bench.py --config $cfg --no-cpu --no-e2e --no-host --steps 20 --warmup 5 > $T/c${cfg}_f$fz.log 2>&1 || exit 1
  done
done
