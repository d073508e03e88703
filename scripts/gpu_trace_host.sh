#!/bin/bash
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_ps.py tests/test_gpu_sbr.py tests/test_golden.py -q -x > gpurun_out/sbrps_pytest.log 2>&1 || exit $?
for c in 4 5; do
JAAD_TRACE_HOST=1 timeout -k 10 300 python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu > gpurun_out/trace_c$c.log 2>&1 || exit $?
done
