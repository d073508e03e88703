#!/bin/bash
# PMC passes (instruction mix, wait states) for each library variant in .tmp/exp on the C2 bench.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
C1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES"
C2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"
C3="SQ_LDS_IDX_ACTIVE SQ_INSTS_FLAT SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE"
for lib in .tmp/exp/lib_*.so; do
  v=$(basename $lib .so); export JAAD_LIB=$PWD/$lib
  for k in 1 2 3; do
    eval C=\$C$k
    bash scripts/gpu_pmc.sh ${v}_p$k "$C" || exit 1
  done
done
grep -h "lc_decode" gpurun_out/pmc/*_p[123].log > gpurun_out/pmc_ab.txt
