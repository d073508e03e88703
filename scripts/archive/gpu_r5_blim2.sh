#!/bin/bash
# Round 5: band limit, second cut (HF stores, decor delay lanes) -- suite, A/B, per-lib kernel traces.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $T/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $T/tests.log; [ $rc -eq 0 ] || exit $rc
for c in 4 5; do
  timeout -k 10 300 python -u scripts/ab_inproc.py $c 6 10 .tmp/exp/lib_base.so .tmp/exp/lib_blim.so .tmp/exp/lib_blim2.so > $T/ab_c$c.log 2>&1 || exit 1
done
for lib in base blim2; do for c in 4 5; do
  JAAD_LIB=$PWD/.tmp/exp/lib_$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof -o ${lib}_c$c --output-format csv -- python3 bench.py --config $c --no-cpu --no-e2e --steps 20 --warmup 5 > $T/prof_${lib}_c$c.log 2>&1 || exit 1
done; done
