#!/bin/bash
# Round 5: LDS / issue counters of the C2 bench command for three LC builds (old kernel, old kernel
# without machine LICM, 6-wave pair kernel).
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
T=$1
P="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
JAAD_LC_PAIR=0 JAAD_LIB=$PWD/.tmp/exp/lib_b.so bash scripts/gpu_pmc.sh ${T}_old "$P" &&
JAAD_LIB=$PWD/.tmp/exp/lib_p6e.so bash scripts/gpu_pmc.sh ${T}_p6e "$P"
