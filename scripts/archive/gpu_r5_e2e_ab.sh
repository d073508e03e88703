#!/bin/bash
# Round 5: e2e (host-buffer) bench legs of C4 / C5 for every .tmp/exp/lib_*.so, alternating
# libs, two rounds.   bash scripts/gpu_r5_e2e_ab.sh TAG
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/$1; mkdir -p $T; export TMPDIR=/tmp
JAAD_LIB=$PWD/.tmp/exp/lib_sets.so timeout -k 10 400 python -u -m pytest tests/test_gpu_host_entry.py tests/test_frame_status.py -m gpu -x -q --timeout 200 --timeout-method thread > $T/parity.log 2>&1
rc=$?; echo "parity rc=$rc" >> $T/parity.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for c in 4 5; do
    for lib in .tmp/exp/lib_*.so; do
      v=$(basename $lib .so)
      JAAD_LIB=$PWD/$lib timeout -k 10 300 python -u bench.py --config $c --no-cpu --no-host --steps 5 --warmup 2 > $T/bench_c${c}_${v}_$r.json 2> $T/bench_c${c}_${v}_$r.err || exit $?
    done
  done
done
