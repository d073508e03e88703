#!/bin/bash
# Round 6: optional GPU tests, then a same-process A/B (scripts/ab_inproc.py) of library builds.
#   bash scripts/gpu_r6_ab.sh TAG "CONFIGS" "PYTEST ARGS or -" LIB[@precision=1] ...
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; C=$2; P=$3; shift 3; mkdir -p $T; export TMPDIR=/tmp
if [ "$P" != "-" ]; then
  timeout -k 10 600 python -u -m pytest $P -m gpu -x -q --timeout 300 --timeout-method thread > $T/tests.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> $T/tests.log; [ $rc -eq 0 ] || exit $rc
fi
for c in $C; do
  timeout -k 10 400 python -u scripts/ab_inproc.py $c 8 20 "$@" > $T/ab_c$c.log 2>&1 || exit $?
done
