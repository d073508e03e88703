#!/bin/bash
# SBR / PS GPU parity (downsampled synthesis included), then C4 / C5 A/B of the library variants
# under .tmp/exp (alternating runs).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sbr.py tests/test_gpu_ps.py tests/test_decoder_api.py tests/test_parse_sbr.py tests/test_jni_glue.py -m gpu -x -v --timeout 300 --timeout-method thread -k "not full" > gpurun_out/sbr_tests.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/sbr_tests.log; [ $rc -eq 0 ] || exit $rc
if ls .tmp/exp/lib_*.so >/dev/null 2>&1; then
timeout -k 10 400 python -u scripts/time_variants.py 4 3 > gpurun_out/sbr_ab.log 2>&1 && \
timeout -k 10 400 python -u scripts/time_variants.py 5 3 >> gpurun_out/sbr_ab.log 2>&1
fi
