#!/bin/bash
# LC kernel per-phase stamp breakdown (JAAD_STAMPS build in .tmp/exp), then the rocprofv3 trace
# and PMC passes of the product library (scripts/gpu_prof.sh TAG).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${1:-r3}
JAAD_LIB=.tmp/exp/lib_s_stamps.so timeout -k 10 200 python -u scripts/stamps.py 2 > gpurun_out/stamps_$TAG.log 2>&1 || exit $?
bash scripts/gpu_prof.sh $TAG
