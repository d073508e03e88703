#!/bin/bash
# C2: LC chunk length sweep (JAAD_CHUNK_FRAMES; 0 = planner default), two passes, kernel ms per batch
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
: > gpurun_out/chunk_sweep.log
for pass in 1 2; do
  for L in 0 24 26 29 32 20; do
    JAAD_CHUNK_FRAMES=$L timeout -k 10 120 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/cs.json 2>/dev/null || exit $?
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/cs.json').read().strip().splitlines()[-1]); print('$L', d['roofline']['kernel_ms'], d['ms_per_step'], d['parity_sample']['max_abs_lsb'])" >> gpurun_out/chunk_sweep.log
  done
done
