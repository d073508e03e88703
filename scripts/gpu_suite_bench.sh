#!/bin/bash
# the GPU suite (every failure listed, up to 20), then the default bench line
#   bash scripts/gpu_suite_bench.sh TAG
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail 20 --timeout 200 --timeout-method thread > $T/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc" >> $T/gpu_suite.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -u bench.py > $T/bench.json 2> $T/bench.err
