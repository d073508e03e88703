#!/bin/bash
# Round 5 close: decorrelator step stamps (profiling build), the one <= 300 s parity soak, then the
# bench lines of C2..C5 (all legs) with the round-5 traffic in current_c*.json.
#   bash scripts/gpu_r5_close.sh TAG SOAK_SECONDS
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
JAAD_LIB=$PWD/.tmp/stamps/lib_stamps.so timeout -k 10 200 python -u scripts/decor_stamps.py > $T/decor_stamps.txt 2>&1 || exit $?
JAAD_SOAK_SEED=17 JAAD_SOAK_SECONDS=$2 timeout -k 10 $(( $2 + 200 )) python -u -m pytest tests/test_gpu_soak.py -m gpu -x -q -s --timeout $(( $2 + 150 )) --timeout-method thread > $T/soak.log 2>&1
rc=$?; echo "soak rc=$rc" >> $T/soak.log; [ $rc -eq 0 ] || exit $rc
for c in 2 3 4 5; do
  timeout -k 10 400 python -u bench.py --config $c > $T/bench_c$c.json 2> $T/bench_c$c.err || exit $?
done
