mkdir -p gpurun_out/fs
for r in 1 2; do for cfg in base nostamp; do
  if [ $cfg = nostamp ]; then export DORA_GPU_REGION_CP_STAMPS=0; else unset DORA_GPU_REGION_CP_STAMPS; fi
  DORA_BENCH_FIRST_PHASES=1 timeout -k 10 120 python -u bench.py --no-ladder --no-cpu-baseline --no-c3 --steps 20 --warmup 5 > gpurun_out/fs/${cfg}_$r.json 2> gpurun_out/fs/${cfg}_$r.err || exit 1
done; done; echo ok
