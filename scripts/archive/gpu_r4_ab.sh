#!/bin/bash
# round 4: the GPU suite on the product library, parity of one variant, then same-call A/B of the
# .tmp/exp variants (scripts/build_variants.py) on the given configs (30 launches each, 3 rounds).
#   bash scripts/gpu_r4_ab.sh TAG VARIANT_FOR_PARITY CONFIG...
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
V=$2; shift 2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $T/gpu_suite.log 2>&1
rc=$?; echo "suite rc=$rc" >> $T/gpu_suite.log
case $rc in 124|134|137|139) exit $rc;; esac
if [ "$V" != "-" ]; then
  JAAD_LIB=$PWD/.tmp/exp/lib_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sbr.py -m gpu -x -q --timeout 200 --timeout-method thread > $T/parity_$V.log 2>&1
  rc=$?; echo "parity rc=$rc" >> $T/parity_$V.log
  case $rc in 124|134|137|139) exit $rc;; esac
fi
for c in "$@"; do timeout -k 10 300 python -u scripts/time_variants.py $c 3 > $T/ab_c$c.log 2>&1 || exit $?; done
