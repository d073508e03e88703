#!/bin/bash
# Round 5: PMC passes of the bench's C2 command for the pair kernel and lc_decode_kernel
# (JAAD_LC_PAIR=0), plus a timing A/B with an ablation build in .tmp/exp/lib_c.so.
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=$1
timeout -k 10 240 python -u scripts/ab_inproc.py 2 4 20 .tmp/exp/lib_a.so .tmp/exp/lib_b.so@JAAD_LC_PAIR=0 .tmp/exp/lib_c.so > gpurun_out/$T.ab.log 2>&1 || exit $?
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
P2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
bash scripts/gpu_pmc.sh ${T}_pair1 "$P1" && bash scripts/gpu_pmc.sh ${T}_pair2 "$P2" || exit $?
JAAD_LC_PAIR=0 bash scripts/gpu_pmc.sh ${T}_old1 "$P1" && JAAD_LC_PAIR=0 bash scripts/gpu_pmc.sh ${T}_old2 "$P2"
