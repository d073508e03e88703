#!/bin/bash
# round 4: synthesis chunks sized from the resident waves -- SBR/PS parity, then kernel traces of
# C4 / C5 with the round-3 fixed 4-frame chunks (JAAD_SYN_FRAMES=4) and with the sized ones
cd "$GRAFT_REPO_ROOT"; T=gpurun_out/r4syn; mkdir -p $T; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ps.py tests/test_gpu_sbr.py tests/test_frame_status.py tests/test_multichannel.py tests/test_cce.py -m gpu -x -q --timeout 300 --timeout-method thread > $T/parity.log 2>&1
rc=$?; echo "parity rc=$rc" >> $T/parity.log; [ $rc -eq 0 ] || exit $rc
for c in 4 5; do
  s=0; [ $c = 5 ] && s=256
  JAAD_SYN_FRAMES=4 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $T/fixed4_c$c -o kt --output-format csv -- python3 scripts/decode_loop.py $c 30 $s > $T/fixed4_c$c.log 2>&1 || exit $?
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $T/sized_c$c -o kt --output-format csv -- python3 scripts/decode_loop.py $c 30 $s > $T/sized_c$c.log 2>&1 || exit $?
done
for c in 4 5; do timeout -k 10 300 python3 bench.py --config $c > $T/bench_c$c.json 2> $T/bench_c$c.err || exit $?; done
