#!/bin/bash
# rocprofv3: kernel trace/stats pass over the bench's own 25 launches, then separate PMC passes
# (never combined with tracing domains).   bash scripts/gpu_prof.sh TAG [CONFIG]
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
export TMPDIR=/tmp
TAG=${1:-r1}
CFG=${2:-2}
B="python3 bench.py --config $CFG --no-cpu --no-e2e --no-host"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/$TAG -o trace --output-format csv -- $B --steps 20 --warmup 5 > gpurun_out/prof/$TAG.bench.log 2>&1
rc=$?; echo "trace rc=$rc" >> gpurun_out/prof/$TAG.bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d gpurun_out/prof/$TAG -o pmc1 --output-format csv -- $B --steps 3 --warmup 1 > gpurun_out/prof/$TAG.pmc1.log 2>&1
rc=$?; echo "pmc1 rc=$rc" >> gpurun_out/prof/$TAG.pmc1.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS -d gpurun_out/prof/$TAG -o pmc2 --output-format csv -- $B --steps 3 --warmup 1 > gpurun_out/prof/$TAG.pmc2.log 2>&1
rc=$?; echo "pmc2 rc=$rc" >> gpurun_out/prof/$TAG.pmc2.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof/$TAG -o pmc3 --output-format csv -- $B --steps 3 --warmup 1 > gpurun_out/prof/$TAG.pmc3.log 2>&1
rc=$?; echo "pmc3 rc=$rc" >> gpurun_out/prof/$TAG.pmc3.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE GRBM_GUI_ACTIVE -d gpurun_out/prof/$TAG -o pmc4 --output-format csv -- $B --steps 3 --warmup 1 > gpurun_out/prof/$TAG.pmc4.log 2>&1
rc=$?; echo "pmc4 rc=$rc" >> gpurun_out/prof/$TAG.pmc4.log
python3 scripts/summarize_prof.py gpurun_out/prof/$TAG $TAG gpurun_out/prof $CFG > gpurun_out/prof/$TAG.summary.log 2>&1
exit $rc
