#!/bin/bash
# PMC passes on the C4 workload, or the config given as $1 (separate passes, no tracing domains).
cd "$GRAFT_REPO_ROOT"; CFG=${1:-4}; mkdir -p gpurun_out/pmc$CFG; export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY -d gpurun_out/pmc$CFG/p1 -o p1 --output-format csv -- python3 bench.py --config $CFG --steps 2 --warmup 1 --no-cpu --no-e2e --no-host > gpurun_out/pmc$CFG/p1.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY -d gpurun_out/pmc$CFG/p2 -o p2 --output-format csv -- python3 bench.py --config $CFG --steps 2 --warmup 1 --no-cpu --no-e2e --no-host > gpurun_out/pmc$CFG/p2.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc$CFG/p3 -o p3 --output-format csv -- python3 bench.py --config $CFG --steps 2 --warmup 1 --no-cpu --no-e2e --no-host > gpurun_out/pmc$CFG/p3.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc$CFG/p4 -o p4 --output-format csv -- python3 bench.py --config $CFG --steps 2 --warmup 1 --no-cpu --no-e2e --no-host > gpurun_out/pmc$CFG/p4.log 2>&1
