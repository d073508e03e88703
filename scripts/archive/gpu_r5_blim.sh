#!/bin/bash
# Round 5: band-limited SBR/PS rows -- GPU suite, same-process A/B (C4, C5), C5 kernel trace + PMC.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp; T=gpurun_out/$1; mkdir -p $T
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $T/tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $T/tests.log; [ $rc -eq 0 ] || exit $rc
for c in 5 4; do
  timeout -k 10 300 python -u scripts/ab_inproc.py $c 6 10 .tmp/exp/lib_base.so .tmp/exp/lib_blim.so > $T/ab_c$c.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $T/prof -o c5 --output-format csv -- python3 bench.py --config 5 --no-cpu --no-e2e --steps 20 --warmup 5 > $T/prof_c5.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $T/prof -o c5f --output-format csv -- python3 bench.py --config 5 --no-cpu --no-e2e --steps 3 --warmup 1 > $T/pmc_c5f.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $T/prof -o c5w --output-format csv -- python3 bench.py --config 5 --no-cpu --no-e2e --steps 3 --warmup 1 > $T/pmc_c5w.log 2>&1
