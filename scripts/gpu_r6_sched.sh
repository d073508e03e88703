#!/bin/bash
# Round 6: machine-scheduler A/B. LSB1 C2/C3 in-process (product vs exp/lib_fast_*), then per-kernel rocprof of
# C4/C5 for the SBR / PS / exact-LC translation units under iterative-ilp.   bash scripts/gpu_r6_sched.sh TAG
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
OUT=gpurun_out/$1; mkdir -p $OUT
P=jaadec_amd/libjaadgpu.so
timeout -k 10 200 python -u scripts/ab_inproc.py 2 16 20 $P@precision=1 exp/lib_fast_max-ilp.so@precision=1 exp/lib_fast_max-memory-clause.so@precision=1 > $OUT/ab_c2.log 2>&1 &&
timeout -k 10 200 python -u scripts/ab_inproc.py 3 12 20 $P@precision=1@hint=1 exp/lib_fast_max-ilp.so@precision=1@hint=1 exp/lib_fast_max-memory-clause.so@precision=1@hint=1 > $OUT/ab_c3.log 2>&1 &&
bash scripts/gpu_r6_ab_prof.sh $1 "4 5" - exp/lib_ps_ilp.so exp/lib_sbr_ilp.so exp/lib_lc_ilp_all.so
