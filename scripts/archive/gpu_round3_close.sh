#!/bin/bash
# Round-3 closing measurements: the whole GPU suite + smoke(), bench lines C2-C5, then the C2 kernel
# trace + PMC passes (scripts/gpu_prof.sh).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash scripts/gpu_all_tests.sh || exit $?
bash scripts/gpu_bench_all.sh || exit $?
bash scripts/gpu_prof.sh ${1:-r3c}
