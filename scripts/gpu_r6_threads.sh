mkdir -p gpurun_out/r6r
for t in 16 12 8 16; do
  JAAD_HOST_THREADS=$t JAAD_TRACE_HOST=1 timeout -k 10 120 python -u bench.py --config 4 --no-cpu --no-e2e --no-host --steps 40 --warmup 5 > gpurun_out/r6r/c4_t$t.json 2> gpurun_out/r6r/c4_t$t.err || exit 1
  JAAD_HOST_THREADS=$t timeout -k 10 120 python -u bench.py --config 5 --no-cpu --no-e2e --no-host --steps 40 --warmup 5 > gpurun_out/r6r/c5_t$t.json 2> gpurun_out/r6r/c5_t$t.err || exit 1
done
