#!/bin/bash
# Round 6: per-kernel A/B by rocprofv3 kernel trace of the bench (C4/C5), product vs exp/ libs, then
# an optional pytest selection first.   bash scripts/gpu_r6_ab_prof.sh TAG "CONFIGS" "PYTEST ARGS or -" lib...
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; CFGS=$2; PYT=$3; shift 3
OUT=gpurun_out/$TAG; mkdir -p $OUT
if [ "$PYT" != "-" ]; then
  timeout -k 10 400 python -u -m pytest $PYT -x -q --timeout 120 --timeout-method thread -m gpu > $OUT/tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $OUT/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for cfg in $CFGS; do
  for lib in jaadec_amd/libjaadgpu.so "$@"; do
    n=$(basename $lib .so)
    JAAD_LIB=$lib timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $OUT/c${cfg}_$n -o trace --output-format csv -- python3 bench.py --config $cfg --no-cpu --no-e2e --no-host --steps 20 --warmup 5 > $OUT/c${cfg}_$n.log 2>&1
    rc=$?; echo "rc=$rc" >> $OUT/c${cfg}_$n.log; [ $rc -eq 0 ] || exit $rc
  done
done
