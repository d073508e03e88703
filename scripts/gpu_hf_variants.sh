#!/bin/bash
# Kernel trace of each .tmp/exp variant on a config (default C4): per-kernel average times.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/hfv; export TMPDIR=/tmp
C=${1:-4}
for lib in .tmp/exp/lib_*.so; do
  n=$(basename $lib .so)
  JAAD_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/hfv/$n -o t --output-format csv -- python3 bench.py --config $C --steps 3 --warmup 1 --no-cpu > gpurun_out/hfv/$n.log 2>&1 || exit $?
  echo "== $n" >> gpurun_out/hfv/summary.txt
  python3 scripts/kstats.py $(find gpurun_out/hfv/$n -name "*kernel_stats.csv" | head -1) >> gpurun_out/hfv/summary.txt
done
