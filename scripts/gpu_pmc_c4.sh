#!/bin/bash
# PMC passes (separate, kernel-trace only) for the SBR kernels of C4.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmc4; export TMPDIR=/tmp
C=${1:-4}
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/pmc4 -o p1 --output-format csv -- python3 bench.py --config $C --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc4/p1.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d gpurun_out/pmc4 -o p2 --output-format csv -- python3 bench.py --config $C --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc4/p2.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE GRBM_GUI_ACTIVE -d gpurun_out/pmc4 -o p3 --output-format csv -- python3 bench.py --config $C --steps 2 --warmup 1 --no-cpu > gpurun_out/pmc4/p3.log 2>&1
