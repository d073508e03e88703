#!/bin/bash
# Round 6: two SQ PMC passes of the bench on config $2, product vs each exp/ lib (per-kernel table:
# scripts/kernel_pmc.py).   bash scripts/gpu_r6_pmc_ab.sh TAG CONFIG lib...
cd "$GRAFT_REPO_ROOT"; export TMPDIR=/tmp
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
B="python3 bench.py --config $CFG --steps 2 --warmup 1 --no-cpu --no-e2e --no-host"
for lib in jaadec_amd/libjaadgpu.so "$@"; do
  n=$(basename $lib .so)
  JAAD_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY -d $OUT/$n/p1 -o p1 --output-format csv -- $B > $OUT/$n.p1.log 2>&1 || exit 1
  JAAD_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $OUT/$n/p2 -o p2 --output-format csv -- $B > $OUT/$n.p2.log 2>&1 || exit 1
  python3 scripts/kernel_pmc.py $OUT/$n > $OUT/$n.table.txt 2>&1
done
